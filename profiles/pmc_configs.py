#!/usr/bin/env python3
"""Per-configuration kernel launches for rocprofv3 (profiles/collect.sh).

Each configuration prepares its batch in HBM, then launches ONE product
kernel `--reps` times through the C ABI.  Every gcs launch is recorded, in
order, in a manifest: the label of the configuration it measures, or "setup"
for the launches that prepare a batch.  profiles/summarize.py pairs the
manifest with the gcs:: dispatches of a rocprofv3 run (same order: one
stream, every launcher launches exactly one kernel) and averages FETCH_SIZE /
WRITE_SIZE / duration per configuration -- per kernel AND per launch size,
which bench.py then looks up for its roofline.traffic.

Labels: <op>_<layout>_<frame_len|imix>_<frames per launch>, e.g.
compute_fixed_1500_4194304 is the TX fill of a C4 shard; step_fixed_* is the
bench step's ONE launch (gcs_step_fixed_dev: the fill of one batch and the
verify of another); split_step_* are the same step as two launches back to
back (the round-5 bench step), each with its own label.

--scrub writes, then reads, 1 GiB (four times the Infinity Cache) between
launches, outside the HIP events, so each launch starts with nothing of its
batch cached and no dirty line of the scrub (bench.py's _scrub).
Timings (HIP events on the launch stream) are printed as one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ALL = ["C1", "C2", "C2x2", "C4", "C4step", "C3", "C2ext", "C2rooms"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default=",".join(ALL))
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--scrub", action="store_true")
    ap.add_argument("--manifest", default="")
    a = ap.parse_args()

    import torch
    from mtcp_amd import gpucsum, synth

    torch.cuda.set_device(0)
    work = torch.cuda.Stream()
    torch.cuda.set_stream(work)
    stream = work.cuda_stream
    ctx = gpucsum.Context(0)
    manifest: list[str] = []
    timings: dict[str, dict] = {}
    scrub_buf = torch.empty(256 << 20, dtype=torch.int32, device="cuda") if a.scrub else None

    def setup(fn, *args, **kw):
        manifest.append("setup")
        fn(*args, stream=stream, **kw)

    def measure(label, fn, bytes_alg):
        # settle: untimed launches of the same kernel (clock ramp)
        for _ in range(3):
            manifest.append("setup")
            fn()
        ms = []
        for _ in range(a.reps):
            if scrub_buf is not None:
                scrub_buf.fill_(len(ms) & 0xFF)
                scrub_buf.sum()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            manifest.append(label)
            fn()
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        med = float(np.median(ms))
        timings[label] = {"median_us": med * 1e3, "min_us": float(min(ms)) * 1e3,
                          "bytes_algorithmic": bytes_alg,
                          "gbs_algorithmic": bytes_alg / (med * 1e-3) / 1e9}
        print(f"{label:36s} {med * 1e3:9.1f} us  {bytes_alg / (med * 1e-3) / 1e9:8.0f} GB/s",
              file=sys.stderr, flush=True)

    def fixed(L, n, ops=("compute", "verify", "step")):
        tx, stride = synth.fixed_frames_device(n, L, seed=0x5EED ^ n ^ L)
        rx = tx.clone()
        setup(ctx.compute_fixed, rx, stride, L, n)
        v = torch.empty(n, dtype=torch.uint8, device="cuda")
        if "compute" in ops:
            measure(f"compute_fixed_{L}_{n}",
                    lambda: ctx.compute_fixed(tx, stride, L, n, stream=stream), n * (L + 4))
        if "verify" in ops:
            measure(f"verify_fixed_{L}_{n}",
                    lambda: ctx.verify_fixed(rx, stride, L, n, v, stream=stream), n * (L + 1))
        if "step" in ops and L > 64:
            measure(f"step_fixed_{L}_{n}",
                    lambda: ctx.step_fixed(tx, stride, L, n, rx, stride, L, n, v, stream=stream),
                    n * (2 * L + 5))
        torch.cuda.synchronize()
        assert int((v != 0).sum()) == 0
        return tx, rx, stride, v

    for c in a.configs.split(","):
        if c == "C1":
            fixed(64, 1 << 20)
        elif c == "C2":
            fixed(1500, 1 << 20)
        elif c == "C2x2":
            fixed(1500, 2 << 20)
        elif c == "C4":
            fixed(1500, 4 << 20)
        elif c == "C4step":
            n, L = 4 << 20, 1500
            tx, stride = synth.fixed_frames_device(n, L, seed=0x5E9 ^ n)
            rx = tx.clone()
            setup(ctx.compute_fixed, rx, stride, L, n)
            v = torch.empty(n, dtype=torch.uint8, device="cuda")
            for _ in range(3):
                manifest.extend(["setup", "setup"])
                ctx.compute_fixed(tx, stride, L, n, stream=stream)
                ctx.verify_fixed(rx, stride, L, n, v, stream=stream)
            ms = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                manifest.extend([f"split_step_compute_fixed_{L}_{n}",
                                 f"split_step_verify_fixed_{L}_{n}"])
                ctx.compute_fixed(tx, stride, L, n, stream=stream)
                ctx.verify_fixed(rx, stride, L, n, v, stream=stream)
                e1.record()
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            med = float(np.median(ms))
            timings[f"split_step_fixed_{L}_{n}"] = {"median_us": med * 1e3,
                                                    "bytes_algorithmic": n * (2 * L + 5)}
            print(f"split_step_fixed_{L}_{n:<16d} {med * 1e3:9.1f} us", file=sys.stderr,
                  flush=True)
            assert int((v != 0).sum()) == 0
            del tx, rx
        elif c == "C2rooms":
            n, L, room = 1 << 20, 1500, 2048
            buf, _ = synth.fixed_frames_device(n, L, stride=room, seed=0x800F)
            off = torch.arange(n, device="cuda", dtype=torch.int64) * room
            ln = torch.full((n,), L, dtype=torch.int16, device="cuda")
            hint = gpucsum.K["GCS_VF_ROOMS"]
            rx = buf.clone()
            setup(ctx.compute, rx, off, ln, n, flags=hint)
            v = torch.empty(n, dtype=torch.uint8, device="cuda")
            measure(f"compute_rooms_{L}_{n}",
                    lambda: ctx.compute(buf, off, ln, n, flags=hint, stream=stream), n * (L + 4))
            measure(f"verify_rooms_{L}_{n}",
                    lambda: ctx.verify(rx, off, ln, n, v, flags=hint, stream=stream), n * (L + 1))
            torch.cuda.synchronize()
            assert int((v != 0).sum()) == 0
            del buf, rx
        elif c == "C3":
            n = 4 << 20
            lens = synth.imix_lengths(n, seed=0x494D)
            buf, off, ln, total = synth.packed_frames_device(lens, seed=0x494D)
            tx = buf.clone()
            setup(ctx.compute, buf, off, ln, n)
            v = torch.empty(n, dtype=torch.uint8, device="cuda")
            nbytes = int(lens.astype(np.int64).sum())
            measure(f"compute_desc_imix_{n}", lambda: ctx.compute(tx, off, ln, n, stream=stream),
                    nbytes + n * 14)
            measure(f"verify_desc_imix_{n}", lambda: ctx.verify(buf, off, ln, n, v, stream=stream),
                    nbytes + n * 11)
            torch.cuda.synchronize()
            assert int((v != 0).sum()) == 0
            del buf, tx
        elif c == "C2ext":
            n, L = 1 << 20, 1500
            buf, stride = synth.fixed_frames_device(n, L, seed=0x8F)
            setup(ctx.compute_fixed, buf, stride, L, n)
            v = torch.empty(n, dtype=torch.uint8, device="cuda")
            h = torch.empty(n, dtype=torch.int32, device="cuda")
            q = torch.empty(n, dtype=torch.int16, device="cuda")
            ctx.set_rss(None, 16, 0)
            measure(f"classify_fixed_{L}_{n}",
                    lambda: ctx.classify_fixed(buf, stride, L, n, v, h, q, stream=stream),
                    n * (L + 7))
            pl = L - 66
            src = torch.randint(0, 256, (n * pl + 64,), dtype=torch.uint8, device="cuda")
            off = torch.arange(n, device="cuda", dtype=torch.int64) * stride
            src_off = torch.arange(n, device="cuda", dtype=torch.int64) * pl
            lens = torch.full((n,), L, dtype=torch.int16, device="cuda")
            st = torch.empty(n, dtype=torch.uint8, device="cuda")
            measure(f"copy_fill_{L}_{n}",
                    lambda: ctx.compute_copy(buf, off, lens, src, src_off, n, st, stream=stream),
                    n * (pl + 66 + L))
            del src, buf
            sb, stride = synth.tcp_streams_device(n, L)
            off = torch.arange(n, device="cuda", dtype=torch.int64) * stride
            setup(ctx.compute, sb, off, lens, n)
            setup(ctx.verify, sb, off, lens, n, v)
            o = torch.empty_like(sb)
            oo = torch.empty(n, dtype=torch.int64, device="cuda")
            ol = torch.empty(n, dtype=torch.int16, device="cuda")
            hd = torch.empty(n, dtype=torch.int32, device="cuda")
            measure(f"gro_{L}_{n}",
                    lambda: ctx.gro(sb, off, lens, v, n, 64, 16384, o, oo, ol, hd, stream=stream),
                    2 * n * L)
            measure(f"gro256_{L}_{n}",      # windows of 256: the FLAT form, 1,024 threads
                    lambda: ctx.gro(sb, off, lens, v, n, 256, 16384, o, oo, ol, hd, stream=stream),
                    2 * n * L)
            del sb, o
        else:
            raise SystemExit(f"unknown config {c}")
        torch.cuda.empty_cache()
    torch.cuda.synchronize()
    ctx.close()
    if a.manifest:
        os.makedirs(os.path.dirname(a.manifest) or ".", exist_ok=True)
        json.dump({"labels": manifest, "scrub": a.scrub, "reps": a.reps}, open(a.manifest, "w"))
    print(json.dumps({"scrub": a.scrub, "timings": timings}), flush=True)


if __name__ == "__main__":
    main()
