#!/usr/bin/env python3
"""Per-burst latency of the host entry points the io_module plugin calls
(gcs_verify_ptrs / gcs_compute_ptrs: frames scattered in pageable host memory,
one pointer per frame like DPDK mbufs of 2048 B data room,
dpdk_module.c:184-193), with direct mode off (DMA copies) and on (the kernel
reads pinned staging over PCIe), the latter on k_desc_mixed (one block per 256
frames) and on the spread k_desc (8 frames per block).  Prints one JSON line.

    python tools/burst_lat.py [reps]
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mtcp_amd import gpucsum, synth  # noqa: E402


def bursts(n, L, seed):
    src, stride = synth.fixed_frames(n, L, seed=seed)
    room = 2048
    mb = np.zeros(n * room, dtype=np.uint8)          # mbuf data rooms
    for i in range(n):
        mb[i * room:i * room + L] = src[i * stride:i * stride + L]
    ptrs = (C.c_void_p * n)(*[mb.ctypes.data + i * room for i in range(n)])
    lens = np.full(n, L, dtype=np.uint16)
    return mb, ptrs, lens


def run(mode_bytes, reps, spread=1):
    os.environ["GCS_DIRECT_MAX_BYTES"] = str(mode_bytes)
    os.environ["GCS_DIRECT_SPREAD"] = str(spread)
    L_ = gpucsum.lib()
    out = {}
    with gpucsum.Context(0, max_frames=1 << 12, max_bytes=16 << 20) as ctx:
        for L in (64, 1500):
            for n in (16, 64, 256, 1024):
                mb, ptrs, lens = bursts(n, L, seed=L * 7 + n)
                v = np.zeros(n, dtype=np.uint8)
                st = np.zeros(n, dtype=np.uint8)
                cs = np.zeros(n, dtype=np.uint32)
                # fill first (on the host frames), then verify
                gpucsum.check(L_.gcs_compute_ptrs(ctx.h, ptrs, lens.ctypes.data, n,
                                                  st.ctypes.data, cs.ctypes.data), "compute")
                res = {}
                for op in ("verify", "compute"):
                    ts = []
                    for _ in range(reps):
                        t0 = time.perf_counter()
                        if op == "verify":
                            rc = L_.gcs_verify_ptrs(ctx.h, ptrs, lens.ctypes.data, n,
                                                    v.ctypes.data, 0)
                        else:
                            rc = L_.gcs_compute_ptrs(ctx.h, ptrs, lens.ctypes.data, n,
                                                     st.ctypes.data, cs.ctypes.data)
                        ts.append(time.perf_counter() - t0)
                        gpucsum.check(rc, op)
                    res[op + "_us"] = float(np.median(ts) * 1e6)
                assert int((v != 0).sum()) == 0 and int((st != 0).sum()) == 0
                res["verdict_sum"] = int(v.sum())
                res["csum_xor"] = int(np.bitwise_xor.reduce(cs))
                out[f"{n}x{L}"] = res
    return out


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dma = run(0, reps)
    mixed = run(1 << 30, reps, spread=0)
    direct = run(1 << 30, reps, spread=1)
    for k in dma:
        assert dma[k]["csum_xor"] == direct[k]["csum_xor"] == mixed[k]["csum_xor"], k
    line = {"what": "per-burst latency of gcs_verify_ptrs / gcs_compute_ptrs, median of "
                    f"{reps} calls, pageable frames in 2048 B rooms",
            "dma_copies": {k: {kk: round(vv, 1) for kk, vv in v.items() if kk.endswith("_us")}
                           for k, v in dma.items()},
            "direct_mixed_kernel": {k: {kk: round(vv, 1) for kk, vv in v.items()
                                        if kk.endswith("_us")} for k, v in mixed.items()},
            "direct": {k: {kk: round(vv, 1) for kk, vv in v.items() if kk.endswith("_us")}
                       for k, v in direct.items()}}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
