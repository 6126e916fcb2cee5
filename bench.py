#!/usr/bin/env python3
"""bench.py -- mTCP software checksum path on MI355X (BASELINE.json metric).

One step = one TX pass (gcs compute: fill iph->check / tcph->check in place,
ip_out.c:143-173, tcp_out.c:323-333) over a TX batch plus one RX pass (gcs
verify: one verdict byte per frame, ip_in.c:21-59, tcp_in.c:1208-1241) over a
separate RX batch, both device-resident in HBM.  Every frame-checksum counts
as one packet: value = (TX frames + RX frames) x N_gpus x steps / time.

Workload: N=1 -> C2, 1M x 1500 B frames per batch at stride
1536; N>1 -> C4, 4M x 1500 B frames per GPU (32M at 8 GPUs), sharded by frame
range with no collective (the only torch.distributed calls are the timing
barrier and the max-over-ranks reduction).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE compact JSON line on rank 0 (the contract's fields, roofline, CPU
baseline, per-GPU rates and one scalar per side configuration, < 6 KB); the
side measurements' full tables go to profiles/bench_extras_last.json.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ("Gpkt/s + GiB/s checksummed (device-resident), 64B & 1500B frames, 1/2/4/8 GPU")
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--frames-per-gpu", type=int, default=0,
                   help="default: 1M at N=1 (C2), 4M at N>1 (C4)")
    p.add_argument("--frame-len", type=int, default=1500)
    p.add_argument("--cpu-seconds", type=float, default=8.0,
                   help="CPU-baseline time budget (rank 0, N=1 only); 0 disables")
    p.add_argument("--cpu-sample", type=int, default=1 << 18,
                   help="frames in the CPU-baseline sample")
    p.add_argument("--settle-s", type=float, default=1.0,
                   help="untimed seconds of the same kernels before the W warmup steps: "
                        "the HBM/GPU clocks take ~10 ms of load to reach steady state "
                        "(DESIGN.md App. A); reported in the JSON line")
    p.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                   help="process group for the timing barrier / max-over-ranks only (nccl = "
                        "RCCL; gloo: rehearsing N>1 ranks on one GPU with GCS_BENCH_DEVICE)")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the side measurements (C1, C3, SURVEY 8f rows, PCIe-inclusive)")
    return p.parse_args()


from mtcp_amd.shard import (aggregate_rate, barrier, env_world, gather_per_rank,  # noqa: E402
                            max_over_ranks)


def dist_setup(args):
    """One process per GPU; torch.distributed (RCCL) only for the timing
    barrier and the max-over-ranks reduction -- no data-path collective."""
    import torch
    import torch.distributed as dist

    world, rank, local = env_world()
    # GCS_BENCH_DEVICE pins every rank to one device: a rehearsal of the N > 1
    # path on a one-GPU box (with --dist-backend gloo; RCCL refuses two ranks
    # on one GPU).  Unset, rank r uses GPU LOCAL_RANK as the driver runs it.
    dev = int(os.environ.get("GCS_BENCH_DEVICE", local if world > 1 else 0))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    return world, rank, dev


def make_batches(ctx, n, frame_len, seed, torch):
    """TX batch (checks zero) and RX batch (= filled TX + 1/1024 frames with one
    byte flipped), both resident in HBM."""
    from mtcp_amd import synth
    tx, stride = synth.fixed_frames_device(n, frame_len, seed=seed)
    stream = torch.cuda.current_stream().cuda_stream
    rx = tx.clone()
    ctx.compute_fixed(rx, stride, frame_len, n, stream=stream)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed ^ 0xBAD)
    pick = torch.nonzero(torch.randint(0, 1024, (n,), device="cuda", generator=g) == 0)[:, 0]
    pos = torch.randint(14, frame_len, (pick.numel(),), device="cuda", generator=g)
    flip = torch.randint(1, 256, (pick.numel(),), device="cuda", generator=g).to(torch.uint8)
    idx = pick * stride + pos
    rx[idx] = rx[idx] ^ flip
    torch.cuda.synchronize()
    return tx, rx, stride, int(pick.numel())


def time_steps(ctx, tx, rx, stride, frame_len, n, steps, warmup, world, torch, settle_s=0.0,
               fused=True):
    """W untimed warmup steps, then exactly K timed steps between a barrier +
    synchronize on both sides.  A step is the TX fill of `tx` and the RX
    verify of `rx`: ONE launch (gcs_step_fixed_dev, fused=True: mTCP's loop
    folds RX and TX each iteration) or the two launches (fused=False).  One
    HIP event per step boundary on the launches' own stream (K + 1 in all,
    nothing between a step's kernels): the fused launch's duration per step.
    Returns (wall seconds, per-step event ms, verdicts)."""
    stream = torch.cuda.current_stream().cuda_stream
    assert stream, "kernels must run on the events' stream"
    verdict = torch.empty(n, dtype=torch.uint8, device="cuda")

    def step():
        if fused:
            ctx.step_fixed(tx, stride, frame_len, n, rx, stride, frame_len, n, verdict,
                           stream=stream)
        else:
            ctx.compute_fixed(tx, stride, frame_len, n, stream=stream)
            ctx.verify_fixed(rx, stride, frame_len, n, verdict, stream=stream)

    if settle_s > 0:
        # bring HBM/GPU clocks to their loaded state: untimed
        # passes of the same kernels, before and separate from the W warmups
        t_end = time.perf_counter() + settle_s
        while time.perf_counter() < t_end:
            for _ in range(10):
                step()
            torch.cuda.synchronize()
    for _ in range(warmup):
        step()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        evs[k].record()
        step()
    evs[steps].record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    step_ms = [evs[k].elapsed_time(evs[k + 1]) for k in range(steps)]
    return t1 - t0, step_ms, verdict


def split_kernels_ms(ctx, tx, rx, stride, frame_len, n, torch, reps=20):
    """After the timed region (untimed for the line): the step's two halves
    as separate launches -- the TX fill and the RX verify, each timed back to
    back with HIP events -- so the per-kernel figures stay on record beside
    the fused step.  The TX fill rewrites the checks it wrote in the step
    (refills), as the round-5 line's per-kernel figures did."""
    stream = torch.cuda.current_stream().cuda_stream
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {}
    for name, fn in (("compute", lambda: ctx.compute_fixed(tx, stride, frame_len, n,
                                                           stream=stream)),
                     ("verify", lambda: ctx.verify_fixed(rx, stride, frame_len, n, v,
                                                         stream=stream))):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / reps
    return out


def pmc_row(label: str):
    """PMC row of one configuration -- kernel AND frames per launch -- from the
    committed rocprofv3 summary (profiles/pmc_summary.json: collect.sh +
    summarize.py, gfx950 FETCH_SIZE x2 correction), or None when that exact
    configuration was not profiled."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        return json.load(open(p))["configs"][label]
    except Exception:
        return None


def step_bytes(n, L):
    """Algorithmic bytes of one step: TX L + 4, RX L + 1 per frame."""
    return n * (L + 4) + n * (L + 1)


def step_frac(n, L, step_ms):
    """Algorithmic GB/s of the fused step launch / the HBM peak."""
    return step_bytes(n, L) / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS


def host_cpus():
    """CPUs this process may run on, ordered for the CPU baseline, and how
    many it may use at once.  The GPU box gives a job a share of a large host:
    sched_getaffinity lists the whole machine, the cgroup's cpu.max bounds
    what runs at once.  Order: one hardware thread per physical core (SMT
    siblings last), round-robin over the L3 domains (CCDs), so N threads get
    N cores' worth of cache and memory links; CPU 0 (interrupts) last."""
    cpus = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except Exception:
        pass
    usable = len(cpus) if quota is None else max(1, min(len(cpus), int(quota)))

    def first_of(path, c):
        try:
            txt = open(f"/sys/devices/system/cpu/cpu{c}/{path}").read().strip()
            return int(txt.replace("-", ",").split(",")[0])
        except Exception:
            return c

    domains: dict[int, list[int]] = {}
    siblings = []
    for c in cpus:
        if first_of("topology/thread_siblings_list", c) != c:
            siblings.append(c)                 # a second hardware thread of a core
            continue
        domains.setdefault(first_of("cache/index3/shared_cpu_list", c), []).append(c)
    order = []
    lists = [sorted(v) for _, v in sorted(domains.items())]
    for k in range(max((len(v) for v in lists), default=0)):
        order += [v[k] for v in lists if k < len(v)]
    order += siblings
    if order and order[0] == 0 and len(order) > 1:
        order = order[1:] + [0]
    return order or cpus, usable, quota


def cpu_baseline(tx, rx, stride, frame_len, budget_s, sample, torch):
    """The reference's own software path (oracle/_ref: mTCP's TCPCalcChecksum +
    ip_fast_csum, reference compile flags) on host cores over a bounded sample
    of the SAME frames; the clean-room port if _ref was never built."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle, RefHarness

    m = min(sample, tx.numel() // stride)
    cpus, usable, quota = host_cpus()
    one = [cpus[0]]
    allc = cpus[:usable]            # spread over cores and L3 domains (host_cpus)
    # The sample is first touched by this thread pinned to the 1-core CPU, so
    # its pages sit on that CPU's memory node, as under `taskset -c <cpu>`
    # (BASELINE.md); the affinity is restored afterwards.
    keep = os.sched_getaffinity(0)
    os.sched_setaffinity(0, set(one))
    try:
        tx_h = tx[: m * stride].cpu().numpy().copy()
        rx_h = rx[: m * stride].cpu().numpy().copy()
    finally:
        os.sched_setaffinity(0, keep)
    kind = "reference" if RefHarness.available() else "port"
    if kind == "reference":
        R = RefHarness()

        def run(buf, compute, pin):
            return R.run_fixed(buf, stride, frame_len, m, compute, cpus=pin)
    else:
        O = Oracle()

        def run(buf, compute, pin):
            if compute:
                return O.compute_fixed(buf, stride, frame_len, m, threads=len(pin), want=False)
            return O.verify_fixed(buf, stride, frame_len, m, threads=len(pin))

    def measure(pin, budget):
        rates = []
        t_start = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            run(tx_h, True, pin)
            run(rx_h, False, pin)
            dt = time.perf_counter() - t0
            rates.append(2 * m / dt)
            if time.perf_counter() - t_start >= budget and len(rates) >= 3:
                break
        return float(np.median(rates)), len(rates)

    r1, reps1 = measure(one, budget_s)
    rmt, repsmt = measure(allc, max(1.0, budget_s / 4))
    try:
        cpu_model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                         if l.startswith("model name"))
    except Exception:
        cpu_model = "unknown"
    pinned = "pinned" if kind == "reference" else "unpinned (port fallback)"
    return {
        "value": r1 / 1e9, "unit": "Gpkt/s", "cores": 1, "kind": kind,
        "sample": f"{m} TX + {m} RX frames of the bench batches ({frame_len} B, stride {stride}),"
                  f" median of {reps1} passes, 1 thread {pinned} to CPU {one[0]}",
        "gib_per_s": r1 * frame_len / 2**30,
        "multi_core": {"value": rmt / 1e9, "unit": "Gpkt/s", "cores": len(allc),
                       "gib_per_s": rmt * frame_len / 2**30, "passes": repsmt,
                       "threads": f"one per usable host core, each {pinned} to its CPU, "
                                  "one per physical core, spread over the L3 domains",
                       "cpus": allc,
                       "affinity_cpus": len(cpus), "cgroup_cpu_quota": quota},
        "cpu_model": cpu_model,
    }


def c1_small_frames(ctx, torch, n=1 << 20, steps=20):
    """C1 side measurement: n x 64 B frames (C1: 1M), IP+TCP verify,
    device-resident.  At 1M the 64 MiB batch is Infinity-Cache resident; 8M
    (512 MiB) is the HBM-resident figure."""
    from mtcp_amd import synth
    L = 64
    buf, stride = synth.fixed_frames_device(n, L, seed=0x6401)
    stream = torch.cuda.current_stream().cuda_stream
    ctx.compute_fixed(buf, stride, L, n, stream=stream)
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    _settle(torch, lambda: ctx.verify_fixed(buf, stride, L, n, v, stream=stream))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    _queue_ahead(torch)
    e0.record()
    for _ in range(steps):
        ctx.verify_fixed(buf, stride, L, n, v, stream=stream)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    assert int((v != 0).sum()) == 0
    out = {"workload": f"{n} x 64B verify, stride 64, back-to-back launches",
           "ms_per_launch": ms, "gpkt_per_s": n / ms / 1e6,
           "gib_per_s": n * L / (ms * 1e-3) / 2**30}
    key = "cache_resident_gbs_algorithmic" if n * stride <= (128 << 20) else \
        "hbm_gbs_algorithmic"
    out[key] = n * (L + 1) / (ms * 1e-3) / 1e9
    # one launch at a time, each after a cache scrub: the HBM-resident figure
    # at this size (the back-to-back rate above reads a cached batch)
    cms = _launch_ms_cold(torch, lambda: ctx.verify_fixed(buf, stride, L, n, v, stream=stream))
    assert int((v != 0).sum()) == 0
    out["cold_ms"] = cms
    out["cold_gpkt_per_s"] = n / cms / 1e6
    out["cold_frac_peak"] = n * (L + 1) / (cms * 1e-3) / 1e9 / HBM_PEAK_GBS
    out["cold_note"] = ("single launches, each after an untimed write + read of 1 GiB "
                        "(4x the Infinity Cache): no line of the batch cached")
    return out


def _settle(torch, fn, seconds=0.25):
    """Untimed launches of `fn` for `seconds`: the side measurements follow the
    CPU baseline, during which the GPU idles and its clocks drop; the first
    ~10 ms of load then run 20-25 % slow (settle phase)."""
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        for _ in range(20):
            fn()
        torch.cuda.synchronize()


def _queue_ahead(torch, cycles=4_000_000):
    """A ~2 ms spin kernel ahead of the timed launches: while the GPU runs it,
    Python enqueues them, so back-to-back kernels of a few us are timed
    without the host's per-launch gaps (which would otherwise be measured)."""
    torch.cuda._sleep(cycles)


def _launch_ms(torch, fn, reps=20, warm=3):
    """Mean HIP-event time of `fn()` launched back to back on the current
    stream, after a settle phase of the same launches."""
    _settle(torch, fn)
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    _queue_ahead(torch)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


SCRUB_BYTES = 1 << 30   # 4x the 256 MB Infinity Cache (MI355X_MICROARCH.md)
_scrub_buf = []


def _scrub(torch):
    """Untimed: write, then read, 1 GiB that no measured kernel touches, so
    neither the L2s nor the Infinity Cache hold any line of the batch -- and
    none of the scrub's own lines is dirty -- when the next launch starts.
    The read pass evicts the write pass's dirty lines (written back here,
    before the timed region), leaving only clean lines behind."""
    if not _scrub_buf:
        _scrub_buf.append(torch.empty(SCRUB_BYTES // 4, dtype=torch.int32, device="cuda"))
    b = _scrub_buf[0]
    b.fill_(int(time.perf_counter_ns() & 0x7FFF))
    return b.sum()   # a device scalar: stays on the stream, no host sync


def _launch_ms_fresh(torch, fn, prep, reps=20, scrub=False):
    """Mean HIP-event time of `fn()` timed launch by launch, with the untimed
    `prep()` before each: a TX fill over frames whose check fields are zero,
    as mTCP hands them over (ip_out.c:153, tcp_out.c:323), instead of a refill
    of the checks it wrote last time (unchanged bytes write back cheaper).
    scrub: after prep() and before the timed launch, `_scrub` the caches
    (cache-cold: prep's zeroed sectors are written back to HBM and evicted,
    so the launch reads and writes every line from and to HBM)."""
    _settle(torch, lambda: (prep and prep(), fn()))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    torch.cuda.synchronize()
    for e0, e1 in evs:
        if prep is not None:
            prep()
        if scrub:
            _scrub(torch)
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    return float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))


def _launch_ms_cold(torch, fn, reps=20):
    """Mean HIP-event time of single launches of `fn()`, each after a cache
    scrub (`_scrub`): no line of its batch is cached when it starts."""
    return _launch_ms_fresh(torch, fn, None, reps=reps, scrub=True)


def c2_max_frame(ctx, torch, n=1 << 20, L=1514):
    """C2 at mTCP's largest frame (1500 B of IP MTU + 14 B Ethernet header,
    SURVEY §8d): same stride 1536, TX fill and RX verify per launch."""
    from mtcp_amd import synth
    stream = torch.cuda.current_stream().cuda_stream
    buf, stride = synth.fixed_frames_device(n, L, stride=1536, seed=0x5EA)
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    cms = _launch_ms(torch, lambda: ctx.compute_fixed(buf, stride, L, n, stream=stream))
    vms = _launch_ms(torch, lambda: ctx.verify_fixed(buf, stride, L, n, v, stream=stream))
    assert int((v != 0).sum()) == 0
    return {"workload": f"{n} x {L}B frames, stride {stride}, TX fill and RX verify per launch",
            "compute_ms": cms, "verify_ms": vms,
            "step_gpkt_per_s": 2 * n / (cms + vms) / 1e6,
            "compute_frac_peak": n * (L + 4) / (cms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "verify_frac_peak": n * (L + 1) / (vms * 1e-3) / 1e9 / HBM_PEAK_GBS}


def c3_imix(ctx, torch, n=4 << 20):
    """C3 side measurement: 4M IMIX frames (64/576/1500 at 7:4:1, pslib 64 B
    packing), descriptor batch in HBM, TX fill and RX verify per launch."""
    from mtcp_amd import synth
    lens = synth.imix_lengths(n, seed=0x494D)
    buf, off, ln, total = synth.packed_frames_device(lens, seed=0x494D)
    stream = torch.cuda.current_stream().cuda_stream
    ctx.compute(buf, off, ln, n, stream=stream)
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    vms = _launch_ms(torch, lambda: ctx.verify(buf, off, ln, n, v, stream=stream))
    cms = _launch_ms(torch, lambda: ctx.compute(buf, off, ln, n, stream=stream))
    assert int((v != 0).sum()) == 0
    chk = torch.cat([off + 24, off + 25, off + 50, off + 51])   # every C3 frame has len >= 64

    def zero_checks():
        buf[chk] = 0

    fms = _launch_ms_fresh(torch, lambda: ctx.compute(buf, off, ln, n, stream=stream),
                           zero_checks)
    # the same with the caches scrubbed between the zeroing and the launch:
    # zero_checks dirties exactly the 64 B sectors the fill then reads and
    # writes (268 MB, about the Infinity Cache's size)
    fcold = _launch_ms_fresh(torch, lambda: ctx.compute(buf, off, ln, n, stream=stream),
                             zero_checks, scrub=True)
    ctx.verify(buf, off, ln, n, v, stream=stream)
    torch.cuda.synchronize()
    assert int((v != 0).sum()) == 0
    vcold = _launch_ms_cold(torch, lambda: ctx.verify(buf, off, ln, n, v, stream=stream))
    assert int((v != 0).sum()) == 0
    nbytes = int(lens.astype(np.int64).sum())
    tx_alg, rx_alg = nbytes + n * 14, nbytes + n * 11
    return {"workload": f"C3: {n} IMIX frames (mean {nbytes / n:.1f} B), {total / 1e9:.2f} GB "
                        "packed at 64 B, descriptor batch",
            "verify_ms": vms, "compute_ms": fms, "compute_refill_ms": cms,
            "compute_ms_cold": fcold, "verify_ms_cold": vcold,
            "compute_note": "compute_ms: check fields zeroed (untimed) before each launch, as "
                            "mTCP hands frames over; compute_ms_cold: the same, with the caches "
                            "scrubbed (1 GiB written + read, untimed) after the zeroing; "
                            "compute_refill_ms: back-to-back refills of the same batch (its "
                            "sector write-back rewrites unchanged bytes); verify_ms_cold: single "
                            "launches after a scrub",
            "verify_gpkt_per_s": n / vms / 1e6, "compute_gpkt_per_s": n / fms / 1e6,
            "verify_hbm_gbs_algorithmic": rx_alg / (vms * 1e-3) / 1e9,
            "compute_hbm_gbs_algorithmic": tx_alg / (fms * 1e-3) / 1e9,
            "verify_frac_peak": rx_alg / (vms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "compute_frac_peak": tx_alg / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "compute_cold_frac_peak": tx_alg / (fcold * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "verify_cold_frac_peak": rx_alg / (vcold * 1e-3) / 1e9 / HBM_PEAK_GBS}


def c2_rooms(ctx, torch, n=1 << 20, L=1500, room=2048):
    """C2's frames one per 2 KiB room (DPDK mbufs, dpdk_module.c:44-49,
    184-193) as a device descriptor batch: RX verify and TX fill per launch
    through the packed stream kernel (no hint: no block streams, every frame
    on its per-frame path) and with the rooms hint (GCS_VF_ROOMS /
    GCS_CF_ROOMS: one 32-lane group per frame, line write-back).  The fills
    are timed over zeroed check fields (fresh, as mTCP hands frames over) and
    as back-to-back refills."""
    from mtcp_amd import synth
    stream = torch.cuda.current_stream().cuda_stream
    buf, stride = synth.fixed_frames_device(n, L, stride=room, seed=0x800F)
    off = torch.arange(n, device="cuda", dtype=torch.int64) * room
    ln = torch.full((n,), L, dtype=torch.int16, device="cuda")
    hint = gpucsum_K()["GCS_VF_ROOMS"]
    rows = buf.view(n, room)
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")

    def zero_checks():
        rows[:, 24:26] = 0
        rows[:, 50:52] = 0

    out = {"workload": f"{n} x {L}B frames in {room} B rooms, descriptor batch, per launch"}
    for name, fl in (("stream", 0), ("rooms", hint)):
        ctx.compute(buf, off, ln, n, st, flags=fl, stream=stream)
        out[f"{name}_verify_ms"] = _launch_ms(
            torch, lambda: ctx.verify(buf, off, ln, n, v, flags=fl, stream=stream))
        assert int((v != 0).sum()) == 0
        out[f"{name}_compute_refill_ms"] = _launch_ms(
            torch, lambda: ctx.compute(buf, off, ln, n, st, flags=fl, stream=stream))
        out[f"{name}_compute_ms"] = _launch_ms_fresh(
            torch, lambda: ctx.compute(buf, off, ln, n, st, flags=fl, stream=stream), zero_checks)
        assert int((st != 0).sum()) == 0
        ctx.verify(buf, off, ln, n, v, stream=stream)
        torch.cuda.synchronize()
        assert int((v != 0).sum()) == 0
        out[f"{name}_verify_frac_peak"] = n * (L + 1) / (out[f"{name}_verify_ms"] * 1e-3) / 1e9 \
            / HBM_PEAK_GBS
        out[f"{name}_compute_frac_peak"] = n * (L + 4) / (out[f"{name}_compute_ms"] * 1e-3) \
            / 1e9 / HBM_PEAK_GBS
    # the fixed-stride kernels over the same rooms (stride = room): what the
    # layout itself costs, without descriptors
    ctx.compute_fixed(buf, room, L, n, stream=stream)
    out["fixed_stride_verify_ms"] = _launch_ms(
        torch, lambda: ctx.verify_fixed(buf, room, L, n, v, stream=stream))
    assert int((v != 0).sum()) == 0
    out["fixed_stride_compute_ms"] = _launch_ms_fresh(
        torch, lambda: ctx.compute_fixed(buf, room, L, n, st, stream=stream), zero_checks)
    assert int((st != 0).sum()) == 0
    del buf
    return out


def rows_8f(ctx, torch, n=1 << 20, L=1500):
    """SURVEY §8f rows 2-4 on C2-shaped data (1M x 1500 B), per launch:
    ICMP flag on TCP traffic, classify (verify + RSS), TX payload copy + fill,
    software LRO.  Each checked for its expected outcome."""
    from mtcp_amd import synth
    stream = torch.cuda.current_stream().cuda_stream
    buf, stride = synth.fixed_frames_device(n, L, seed=0x8F)
    ctx.compute_fixed(buf, stride, L, n, stream=stream)
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {}
    ms = _launch_ms(torch, lambda: ctx.verify_fixed(buf, stride, L, n, v, stream=stream))
    out["verify_ms"] = ms
    ms = _launch_ms(torch, lambda: ctx.verify_fixed(buf, stride, L, n, v,
                                                    flags=gpucsum_K()["GCS_VF_ICMP"],
                                                    stream=stream))
    out["verify_icmp_flag_ms"] = ms
    h = torch.empty(n, dtype=torch.int32, device="cuda")
    q = torch.empty(n, dtype=torch.int16, device="cuda")
    ctx.set_rss(None, 16, 0)
    ms = _launch_ms(torch, lambda: ctx.classify_fixed(buf, stride, L, n, v, h, q, stream=stream))
    ctx.set_rss(None, 1, 0)
    assert int((v != 0).sum()) == 0 and int((q < 0).sum()) == 0 and int((q >= 16).sum()) == 0
    out["classify_ms"] = ms
    out["classify_gpkt_per_s"] = n / ms / 1e6
    # copy + fill: payloads from a contiguous send buffer into the frames
    pl = L - 66
    src = torch.randint(0, 256, (n * pl + 64,), dtype=torch.uint8, device="cuda")
    off = torch.arange(n, device="cuda", dtype=torch.int64) * stride
    src_off = torch.arange(n, device="cuda", dtype=torch.int64) * pl
    lens = torch.full((n,), L, dtype=torch.int16, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    ms = _launch_ms(torch, lambda: ctx.compute_copy(buf, off, lens, src, src_off, n, st,
                                                    stream=stream))
    assert int((st != 0).sum()) == 0
    ctx.verify_fixed(buf, stride, L, n, v, stream=stream)
    torch.cuda.synchronize()
    assert int((v != 0).sum()) == 0
    out["copy_fill_ms"] = ms
    out["copy_fill_gbs_algorithmic"] = n * (pl + 66 + L) / (ms * 1e-3) / 1e9
    del src, buf
    # software LRO: 16 flows in runs of 8, windows of 64
    sb, stride = synth.tcp_streams_device(n, L)
    off = torch.arange(n, device="cuda", dtype=torch.int64) * stride
    ctx.compute(sb, off, lens, n, stream=stream)
    ctx.verify(sb, off, lens, n, v, stream=stream)
    o = torch.empty_like(sb)
    oo = torch.empty(n, dtype=torch.int64, device="cuda")
    ol = torch.empty(n, dtype=torch.int16, device="cuda")
    hd = torch.empty(n, dtype=torch.int32, device="cuda")
    ms = _launch_ms(torch, lambda: ctx.gro(sb, off, lens, v, n, 64, 16384, o, oo, ol, hd,
                                           stream=stream))
    heads = int((ol != 0).sum())
    assert heads == n // 8
    out["lro_ms"] = ms
    out["lro_merged_frames"] = heads
    out["lro_gbs_algorithmic"] = 2 * n * L / (ms * 1e-3) / 1e9
    out["lro_frac_peak"] = 2 * n * L / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    # windows of 256 frames (an ENABLELRO DPDK build's larger bursts,
    # dpdk_module.c:44-48): the FLAT form over 1,024-thread blocks (round 5)
    ms = _launch_ms(torch, lambda: ctx.gro(sb, off, lens, v, n, 256, 16384, o, oo, ol, hd,
                                           stream=stream))
    assert int((ol != 0).sum()) == n // 8
    out["lro_w256_ms"] = ms
    out["lro_w256_frac_peak"] = 2 * n * L / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    out["workload"] = (f"{n} x {L} B frames; RSS 16 queues; copy+fill {pl} B payloads from a "
                       "contiguous send buffer; LRO 16 flows in runs of 8, windows of 64 "
                       "(lro_w256: windows of 256)")
    return out


def tx_write_mode(n, stride):
    """The TX fill's write-back for a fixed-stride batch, as the library picks
    it (gcs_kernels.hip launch_fixed): whole 128 B lines while n x 128 B fits
    GCS_TX_LINE_WB_MB (default 128 MiB, inside the Infinity Cache), else lines
    for that many frames and non-temporal 64 B sectors holding the check
    fields for the rest (GCS_TX_HYBRID)."""
    mb = int(os.environ.get("GCS_TX_LINE_WB_MB", "128"))
    if stride % 128:
        return "sector"
    if n * 128 <= (mb << 20):
        return "line"
    hy = os.environ.get("GCS_TX_HYBRID", "nt")
    if hy in ("nt", "sc1"):
        return f"line for the first {(mb << 20) // 128} frames, {hy} sectors after"
    return "sector"


def c2_sector_wb(ctx, torch, tx, stride, L, n):
    """The C2 TX fill with sector write-back forced (GCS_CF_SECTOR_WB): what
    the headline's fill costs without the whole-line write-back its 1M-frame
    batch qualifies for."""
    stream = torch.cuda.current_stream().cuda_stream
    flag = gpucsum_K()["GCS_CF_SECTOR_WB"]
    ms = _launch_ms(torch, lambda: ctx.compute_fixed(tx, stride, L, n, flags=flag, stream=stream))
    line_ms = _launch_ms(torch, lambda: ctx.compute_fixed(tx, stride, L, n, stream=stream))
    return {"workload": f"{n} x {L}B TX fill, stride {stride}, per launch",
            "sector_compute_ms": ms,
            "sector_frac_peak": n * (L + 4) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "line_compute_ms": line_ms,
            "line_frac_peak": n * (L + 4) / (line_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}


def c2_fresh_cold(ctx, torch, tx, stride, L, n):
    """The C2 TX fill over check fields zeroed before each launch (as mTCP
    hands frames over, ip_out.c:153, tcp_out.c:244, 323), with the caches
    scrubbed between the zeroing and the timed launch (`_scrub`), in the
    library's default write-back and with sector write-back forced; and the
    RX verify as single scrubbed launches."""
    stream = torch.cuda.current_stream().cuda_stream
    rows = tx.view(n, stride)

    def zero_checks():
        rows[:, 24:26] = 0      # iph->check (ETH 14 + 10)
        rows[:, 50:52] = 0      # tcph->check (ETH 14 + IP 20 + 16)

    flag = gpucsum_K()["GCS_CF_SECTOR_WB"]
    dflt = _launch_ms_fresh(torch, lambda: ctx.compute_fixed(tx, stride, L, n, stream=stream),
                            zero_checks, scrub=True)
    sect = _launch_ms_fresh(torch, lambda: ctx.compute_fixed(tx, stride, L, n, flags=flag,
                                                             stream=stream),
                            zero_checks, scrub=True)
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    vms = _launch_ms_cold(torch, lambda: ctx.verify_fixed(tx, stride, L, n, v, stream=stream))
    assert int((v != 0).sum()) == 0
    return {"workload": f"{n} x {L}B, stride {stride}: TX fill of zeroed check fields and RX "
                        "verify, single launches, each after a cache scrub",
            "compute_ms": dflt, "tx_write_mode": tx_write_mode(n, stride),
            "compute_frac_peak": n * (L + 4) / (dflt * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "sector_compute_ms": sect,
            "sector_frac_peak": n * (L + 4) / (sect * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "verify_ms": vms,
            "verify_frac_peak": n * (L + 1) / (vms * 1e-3) / 1e9 / HBM_PEAK_GBS}


def c4_shard(ctx, torch, steps, warmup, settle_s, n=4 << 20, L=1500):
    """The N > 1 per-GPU workload on this one GPU: a C4 shard of 4M x 1500 B
    frames, the same fused TX + RX step, settle, warmup and timing as the main
    line (time_steps), so a SCALE curve's per-GPU rate can be read against
    it; the step's two halves as separate launches beside it."""
    tx, rx, stride, nbad = make_batches(ctx, n, L, 0x6D746370, torch)
    el, sl, verdict = time_steps(ctx, tx, rx, stride, L, n, steps, warmup, 1, torch, settle_s)
    bad = int((verdict != 0).sum())
    assert bad == nbad, (bad, nbad)
    sms = float(np.mean(sl))
    split = split_kernels_ms(ctx, tx, rx, stride, L, n, torch)
    tms, rms = split["compute"], split["verify"]
    prow = pmc_row(f"step_fixed_{L}_{n}")
    del tx, rx
    return {"workload": f"C4 shard: {n} x {L}B frames, TX fill + RX verify per step (one launch)",
            "gpkt_per_s": 2 * n * steps / el / 1e9, "ms_per_step": el / steps * 1e3,
            "step_kernel_ms": sms, "compute_ms": tms, "verify_ms": rms,
            "tx_write_mode": tx_write_mode(n, stride),
            "roofline": {"kernel": "step (fill + verify, one launch)",
                         "achieved": step_bytes(n, L) / (sms * 1e-3) / 1e9,
                         "frac": step_frac(n, L, sms),
                         "traffic": prow["hbm_bytes_per_launch"] if prow else None,
                         "traffic_source": (f"profiles/pmc_summary.json configs[step_fixed_"
                                            f"{L}_{n}]" if prow else None)},
            "verify_frac": n * (L + 1) / (rms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "compute_frac": n * (L + 4) / (tms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "corrupted_frames_detected": bad}


def gpucsum_K():
    from mtcp_amd import gpucsum
    return gpucsum.K


def pcie_inclusive(gcs, torch, frame_len=1500, n=1 << 20):
    """Host-resident frames through the host entry points: gcs_verify (H2D of
    the frames, kernel, D2H of 1 B verdicts) and gcs_compute (H2D, kernel, D2H
    of 4 B checks, written back into the host frames).  Two host layouts:
    pinned (gcs_host_alloc: one DMA per staging slot, no host copy) and
    pageable (gathered into pinned staging by GCS_GATHER_THREADS threads).
    Reported beside the device-resident number, never as `value`."""
    from mtcp_amd import synth
    src, stride = synth.fixed_frames(n, frame_len, seed=77)
    off = np.arange(n, dtype=np.uint64) * stride
    lens = np.full(n, frame_len, dtype=np.uint16)
    pinned = gcs.PinnedBuffer(src.nbytes)
    pinned.array[:] = src
    out = {"workload": f"{n} x {frame_len}B frames in host memory, stride {stride}",
           "pcie": "H2D frames + D2H results, 2 staging slots x 48 MiB"}
    with gcs.Context(torch.cuda.current_device(), max_frames=1 << 16, max_bytes=96 << 20) as c:
        for name, buf in (("pinned", pinned.array), ("pageable", src)):
            c.compute_host(buf, off, lens)
            for op in ("verify", "compute"):
                fn = c.verify_host if op == "verify" else c.compute_host
                fn(buf, off, lens)
                reps, t0 = 3, time.perf_counter()
                for _ in range(reps):
                    r = fn(buf, off, lens)
                dt = (time.perf_counter() - t0) / reps
                codes = r if op == "verify" else r[0]
                assert int((codes != 0).sum()) == 0
                out[f"{op}_{name}"] = {"gpkt_per_s": n / dt / 1e9,
                                       "gib_per_s": n * frame_len / dt / 2**30,
                                       "gb_per_s_h2d": n * stride / dt / 1e9}
    pinned.free()
    return out


def plugin_bursts(gcs, reps=300):
    """Per-call latency of the entry points the io_module plugin calls on an
    mTCP burst (gcs_verify_ptrs / gcs_compute_ptrs in recv_pkts / send_pkts):
    64 frames, each in its own 2048 B room as DPDK mbufs hold them
    (dpdk_module.c:76, 184-193).  Modes:
      pageable_direct     rooms in pageable memory: gathered into pinned
                          staging, one kernel launch + event wait per call
      pageable_server     the same, served by the resident burst grid
      registered_direct   rooms registered with gcs_host_register (an mbuf
                          pool would be): read and filled in place over PCIe
      registered_server   in place AND served by the resident grid
    Timed in C (tools/libburst_timer.so, clock_gettime per call) when built,
    else from Python (adds the interpreter's call overhead)."""
    import ctypes as C
    from mtcp_amd import synth
    L_ = gcs.lib()
    tpath = os.path.join(ROOT, "tools", "libburst_timer.so")
    T = C.CDLL(tpath) if os.path.exists(tpath) else None
    out = {"workload": "64-frame bursts (mTCP MAX_PKT_BURST) in 2048 B rooms, median of "
                       f"{reps} calls",
           "timer": "C clock_gettime per call" if T else "python perf_counter per call"}
    n = 64
    rooms = np.zeros(n * 2048 + 4096, dtype=np.uint8)
    base = (-rooms.ctypes.data) % 4096               # page-aligned rooms (registrable)
    mb = rooms[base:base + n * 2048]
    for mode in ("pageable_direct", "pageable_server", "registered_direct",
                 "registered_server"):
        registered = mode.startswith("registered")
        if registered:
            gcs.check(L_.gcs_host_register(mb.ctypes.data, mb.nbytes), "register")
        res = {}
        try:
            with gcs.Context(0, max_frames=1 << 12, max_bytes=16 << 20) as ctx:
                if mode.endswith("server"):
                    ctx.set_burst_server(True)
                for L in (64, 1500):
                    src, stride = synth.fixed_frames(n, L, seed=L)
                    for i in range(n):
                        mb[i * 2048:i * 2048 + L] = src[i * stride:i * stride + L]
                    ptrs = (C.c_void_p * n)(*[mb.ctypes.data + i * 2048 for i in range(n)])
                    lens = np.full(n, L, dtype=np.uint16)
                    v = np.zeros(n, dtype=np.uint8)
                    st = np.zeros(n, dtype=np.uint8)
                    cs = np.zeros(n, dtype=np.uint32)
                    r = {}
                    for op in ("compute", "verify"):
                        fn = L_.gcs_verify_ptrs if op == "verify" else L_.gcs_compute_ptrs
                        outp = v if op == "verify" else st
                        extra = None if op == "verify" else cs.ctypes.data
                        if T is not None:
                            us = np.zeros(reps, dtype=np.float64)
                            gcs.check(T.bt_run(C.cast(fn, C.c_void_p), ctx.h, ptrs,
                                               C.c_void_p(lens.ctypes.data), C.c_uint32(n),
                                               C.c_void_p(outp.ctypes.data), C.c_void_p(extra),
                                               C.c_uint32(reps), C.c_void_p(us.ctypes.data)),
                                      op)
                            ts = us
                        else:
                            ts = []
                            for _ in range(reps):
                                t0 = time.perf_counter()
                                rc = (fn(ctx.h, ptrs, lens.ctypes.data, n, v.ctypes.data, 0)
                                      if op == "verify" else
                                      fn(ctx.h, ptrs, lens.ctypes.data, n, st.ctypes.data,
                                         cs.ctypes.data))
                                ts.append((time.perf_counter() - t0) * 1e6)
                                gcs.check(rc, op)
                        r[op + "_us"] = float(np.median(ts))
                    assert int((v != 0).sum()) == 0 and int((st != 0).sum()) == 0
                    res[f"64x{L}B"] = r
        finally:
            if registered:
                gcs.check(L_.gcs_host_unregister(mb.ctypes.data), "unregister")
        out[mode] = res
    return out


def plugin_threads():
    """Bursts from several mTCP-like threads per GPU (tools/server_scaling.py,
    child processes with HIP's default hardware queues, as the plugin runs):
    one thread per ring (64-frame IMIX fill + verify per iteration) at 1 / 8 /
    12 / 16 threads (and 24 for `shipped`), and T threads each driving R rings with async posts
    (rings_TxR: up to 24 hot rings with only 4 CPUs busy, so the CPU quota
    does not confound the GPU side).  `shipped`: the grid as it ships, per call
    and post -> done; `counters`: the build with phase counters
    (GCS_SERVER_COUNTERS=1), which adds the GPU serving time (gpu_span_us:
    first serving block saw the request -> last one's records stored), its
    per-block phases, and post -> done split into the wait before the GPU saw
    the request, that span, and the way back.  `pinned`: the shipped grid with
    each thread pinned to one CPU (MT_PIN=1), as mTCP pins its threads
    (core.c:1153-1245)."""
    import subprocess
    out = {}
    for name, prof, pin in (("shipped", "0", "0"), ("counters", "1", "0"), ("pinned", "0", "1")):
        # the shipped grid also at 24 threads: more mTCP threads than the box's
        # 16-CPU quota (VERDICT r05 #5's second point)
        env = dict(os.environ, SS_PROF=prof,
                   SS_THREADS="1,8,12,16,24" if name == "shipped" else "1,8,12,16",
                   SS_RINGS="4x2,4x4,4x6", MT_PIN=pin)
        try:
            r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "server_scaling.py")],
                               capture_output=True, text=True, timeout=240, env=env)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            if prof == "0":
                d = drop_zero_counters(d)
            out[name] = d
        except Exception as e:   # a side measurement: report, never fail the bench line
            out[name] = {"error": repr(e)[:200]}
    return out


def drop_zero_counters(series):
    """A series run without the counting grid reports its GPU-side phase
    fields as 0: keep only the fields it measured."""
    out = {}
    for k, v in series.items():
        if isinstance(v, dict):
            v = {kk: vv for kk, vv in v.items() if not (isinstance(vv, float) and vv == 0.0)}
        out[k] = v
    return out


def plugin_rx_async():
    """How long the RX path keeps the mTCP thread inside the plugin per 64 x
    1500 B burst, verifying the burst as one batch or as you go
    (GPUCSUM_RX_GROUP), under the reference's own RX code (ProcessPacket per
    frame); the software path alongside (tools/rx_async_probe.py, child
    process)."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rx_async_probe.py")],
                           capture_output=True, text=True, timeout=240)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:   # a side measurement: report, never fail the bench line
        return {"error": repr(e)[:200]}


def server_poll_cost():
    """What idle burst-server rings cost the PCIe link (tools/poll_cost.py,
    child process): the pinned verify's rate while 0, 8 and 12 other
    contexts keep their rings of the process's grid alive with one 1-frame
    burst every ~200 us."""
    import subprocess
    env = dict(os.environ, PC_KS="0,8,12,0")
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "poll_cost.py")], env=env,
                           capture_output=True, text=True, timeout=180)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        quiet = d["K0"]["gib_per_s"]
        for k in ("K8", "K12"):
            d[k]["loss_vs_quiet"] = round(1 - d[k]["gib_per_s"] / quiet, 4)
        return d
    except Exception as e:   # a side measurement: report, never fail the bench line
        return {"error": repr(e)[:200]}


def plugin_tx_async():
    """How long send_pkts blocks an mTCP-shaped TX loop per 64 x 1500 B burst,
    with the plugin filling frames as mTCP completes them (GPUCSUM_TX_GROUP)
    and without; the software path alongside (tools/tx_async_probe.py, child
    process)."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "tx_async_probe.py")],
                           capture_output=True, text=True, timeout=240)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:   # a side measurement: report, never fail the bench line
        return {"error": repr(e)[:200]}


EXTRAS_PATH = os.path.join(ROOT, "profiles", "bench_extras_last.json")
LINE_MAX_BYTES = 6144   # the driver parses ONE stdout line; round 5's 29 KB was not parsed


def _dig(d, *keys):
    for k in keys:
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return round(d, 4) if isinstance(d, float) else d


def side_scalars(line):
    """One scalar per side configuration (C1, C3, C4, rooms, SURVEY §8f rows,
    PCIe-inclusive, plugin bursts) for the compact line; the full tables go
    to EXTRAS_PATH."""
    g = lambda *ks: _dig(line, *ks)  # noqa: E731
    s = {
        "c1_64B_ms": g("c1_64B", "ms_per_launch"),
        "c1_64B_cold_ms": g("c1_64B", "cold_ms"),
        "c1_64B_cold_frac": g("c1_64B", "cold_frac_peak"),
        "c1_64B_8M_gpkt_per_s": g("c1_64B_8M", "gpkt_per_s"),
        "c2_sector_wb_frac": g("c2_sector_wb", "sector_frac_peak"),
        "c2_fresh_cold_compute_frac": g("c2_fresh_cold", "compute_frac_peak"),
        "c2_fresh_cold_verify_frac": g("c2_fresh_cold", "verify_frac_peak"),
        "c2_1514B_step_gpkt_per_s": g("c2_1514B", "step_gpkt_per_s"),
        "c3_fill_ms": g("c3_imix", "compute_ms"),
        "c3_verify_ms": g("c3_imix", "verify_ms"),
        "c3_fill_frac": g("c3_imix", "compute_frac_peak"),
        "c3_verify_frac": g("c3_imix", "verify_frac_peak"),
        "c3_fill_cold_frac": g("c3_imix", "compute_cold_frac_peak"),
        "c4_ms_per_step": g("c4_shard", "ms_per_step"),
        "c4_gpkt_per_s": g("c4_shard", "gpkt_per_s"),
        "c4_compute_frac": g("c4_shard", "compute_frac"),
        "c4_verify_frac": g("c4_shard", "verify_frac"),
        "rooms_verify_ms": g("c2_rooms", "rooms_verify_ms"),
        "rooms_fill_ms": g("c2_rooms", "rooms_compute_ms"),
        "lro_w64_ms": g("rows_8f", "lro_ms"),
        "lro_w256_ms": g("rows_8f", "lro_w256_ms"),
        "copy_fill_ms": g("rows_8f", "copy_fill_ms"),
        "classify_ms": g("rows_8f", "classify_ms"),
        "pcie_pinned_verify_gib_per_s": g("pcie_inclusive", "verify_pinned", "gib_per_s"),
        "pcie_pinned_fill_gib_per_s": g("pcie_inclusive", "compute_pinned", "gib_per_s"),
        "pcie_pageable_verify_gib_per_s": g("pcie_inclusive", "verify_pageable", "gib_per_s"),
        "burst_registered_server_verify_us": g("plugin_bursts", "registered_server", "64x1500B",
                                               "verify_us"),
        "burst_pageable_direct_verify_us": g("plugin_bursts", "pageable_direct", "64x1500B",
                                             "verify_us"),
        "burst_registered_direct_verify_us": g("plugin_bursts", "registered_direct", "64x1500B",
                                               "verify_us"),
        "rx_async_registered_blocked_us": g("plugin_rx_async", "registered_group0",
                                            "blocked_us_median"),
        "rx_async_software_blocked_us": g("plugin_rx_async", "software_path_registered",
                                          "blocked_us_median"),
        "tx_async_registered_send_pkts_us": g("plugin_tx_async", "registered_groupdefault",
                                              "send_pkts_us_median"),
        "threads16_shipped_us": g("plugin_threads", "shipped", "threads_16", "us_per_call"),
        "threads16_pinned_us": g("plugin_threads", "pinned", "threads_16", "us_per_call"),
        "threads24_shipped_us": g("plugin_threads", "shipped", "threads_24", "us_per_call"),
        "threads24_shipped_us": g("plugin_threads", "shipped", "threads_24", "us_per_call"),
    }
    return {k: v for k, v in s.items() if v is not None}


def compact_line(line, extras_path=None):
    """The ONE JSON line the driver parses: the contract's fields, the
    roofline and CPU baseline, per-GPU rates and one scalar per side
    configuration, well under LINE_MAX_BYTES.  The full side tables are in
    `extras_path` (written beside it)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "gib_per_s",
            "settle_s", "corrupted_frames_detected")
    out = {k: line[k] for k in keep if k in line}
    rf = line.get("roofline", {})
    out["roofline"] = {k: rf[k] for k in ("bound", "kernel", "achieved", "peak", "unit", "frac",
                                          "traffic", "traffic_source",
                                          "bytes_per_launch_algorithmic", "avg_launch_ms",
                                          "tx_write_mode") if k in rf}
    if "kernels_ms" in line:
        out["kernels_ms"] = {k: line["kernels_ms"][k] for k in ("step", "compute", "verify")
                             if k in line["kernels_ms"]}
    cb = line.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample",
                                                  "gib_per_s", "cpu_model") if k in cb}
        mc = cb.get("multi_core")
        if mc:
            out["cpu_baseline"]["multi_core"] = {k: mc[k] for k in ("value", "unit", "cores",
                                                                    "gib_per_s") if k in mc}
    out["per_gpu"] = [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in p.items()
                       if k in ("rank", "device", "gpkt_per_s", "frac_peak", "step_us",
                                "bad_frames_detected", "corrupted_frames")}
                      for p in line.get("per_gpu", [])]
    side = side_scalars(line)
    if side:
        out["side"] = side
    if extras_path:
        out["extras_file"] = os.path.relpath(extras_path, ROOT)
    return out


def main():
    args = parse()
    import torch
    from mtcp_amd import gpucsum

    world, rank, local = dist_setup(args)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    n = args.frames_per_gpu or ((1 << 20) if world == 1 else (1 << 22))
    L = args.frame_len
    ctx = gpucsum.Context(local)
    # A dedicated torch stream: its handle is non-NULL, so the kernels run on
    # exactly the stream the HIP events are recorded on (a NULL stream
    # argument would select the context's own stream).
    work = torch.cuda.Stream()
    torch.cuda.set_stream(work)
    tx, rx, stride, nbad = make_batches(ctx, n, L, 0x6D746370 ^ rank, torch)

    elapsed, step_list, verdict = time_steps(ctx, tx, rx, stride, L, n, args.steps, args.warmup,
                                             world, torch, args.settle_s)
    step_ms = float(np.mean(step_list))
    bad_seen = int((verdict != 0).sum())
    if bad_seen != nbad:
        raise SystemExit(f"rank {rank}: verify flagged {bad_seen} frames, {nbad} corrupted")
    # after the timed region: the step's halves as separate launches, on record
    split = split_kernels_ms(ctx, tx, rx, stride, L, n, torch)
    red_dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    t = max_over_ranks(world, elapsed, device=red_dev)
    per = gather_per_rank(world, [float(rank), float(local), elapsed, step_ms, split["compute"],
                                  split["verify"], float(bad_seen), float(nbad)], device=red_dev)

    rate = aggregate_rate(2 * n, world, args.steps, t)   # TX fills + RX verifies, all ranks
    value = rate / 1e9
    gib = rate * L / 2**30
    # the dominant kernel is the step's one launch (gcs_step_fixed_dev): its
    # algorithmic bytes over its HIP-event time per step
    kbytes = step_bytes(n, L)
    achieved = kbytes / (step_ms * 1e-3) / 1e9
    prow = pmc_row(f"step_fixed_{L}_{n}")
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "Gpkt/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic (seeded mTCP-shaped Eth/IPv4/TCP frames generated in HBM)",
        "config": {
            "workload": ("C2: 1M x 1500B frames, TX fill + RX verify per step" if world == 1
                         and n == (1 << 20) and L == 1500 else
                         f"C4 shard: {n} x {L}B frames per GPU, TX fill + RX verify per step"),
            "frames_per_gpu": n, "frame_len": L, "stride": stride,
            "step": "one launch per step (gcs_step_fixed_dev: the TX batch's fill and the RX "
                    "batch's verify)",
            "parallelism": f"frame-shard x{world} (no collective)",
        },
        "gib_per_s": gib,
        "roofline": {
            "bound": "hbm",
            "kernel": f"step of {n} + {n} x {L}B: " + (prow["kernel"] if prow else
                                                       "k_fixed_step (fill + verify)"),
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            # HBM bytes per launch of THIS configuration (kernel and frames per
            # launch) from rocprofv3 PMC; null when it was not profiled
            "traffic": prow["hbm_bytes_per_launch"] if prow else None,
            "traffic_source": (f"profiles/pmc_summary.json configs[step_fixed_{L}_{n}]"
                               if prow else None),
            "bytes_per_launch_algorithmic": kbytes, "avg_launch_ms": step_ms,
            "tx_write_mode": tx_write_mode(n, stride),
        },
        # the step's halves as separate launches (after the timed region)
        "kernels_ms": {"step": step_ms, "compute": split["compute"], "verify": split["verify"],
                       "step_first_last": [step_list[0], step_list[-1]],
                       "compute_frac": n * (L + 4) / (split["compute"] * 1e-3) / 1e9 /
                       HBM_PEAK_GBS,
                       "verify_frac": n * (L + 1) / (split["verify"] * 1e-3) / 1e9 /
                       HBM_PEAK_GBS},
        # per GPU, like mTCP's per-thread NETSTAT (core.c:189-218): each rank's
        # own rate, its step launch's fraction of peak and bad-frame count
        "per_gpu": [{"rank": int(r), "device": int(d), "gpkt_per_s": 2 * n * args.steps / e / 1e9,
                     "gib_per_s": 2 * n * args.steps * L / e / 2**30,
                     "step_us": sm * 1e3, "compute_us": c * 1e3, "verify_us": v * 1e3,
                     "frac_peak": step_frac(n, L, sm),
                     "bad_frames_detected": int(b), "corrupted_frames": int(nb)}
                    for r, d, e, sm, c, v, b, nb in per],
        "settle_s": args.settle_s,
        "corrupted_frames_detected": bad_seen,
    }
    if rank == 0 and world == 1:
        def side(key, fn):
            """A side measurement: its failure is reported in the line, never
            allowed to cost the line itself (printed after all of them)."""
            try:
                line[key] = fn()
            except Exception as e:   # noqa: BLE001
                line[key] = {"error": repr(e)[:300]}
            torch.cuda.empty_cache()

        if args.cpu_seconds > 0:
            side("cpu_baseline", lambda: cpu_baseline(tx, rx, stride, L, args.cpu_seconds,
                                                      args.cpu_sample, torch))
        if not args.no_extras:
            side("c2_sector_wb", lambda: c2_sector_wb(ctx, torch, tx, stride, L, n))
            if "sector_frac_peak" in line["c2_sector_wb"]:
                line["roofline"]["sector_wb_frac"] = line["c2_sector_wb"]["sector_frac_peak"]
            side("c2_fresh_cold", lambda: c2_fresh_cold(ctx, torch, tx, stride, L, n))
            if "compute_frac_peak" in line["c2_fresh_cold"]:
                line["roofline"]["fresh_cold_frac"] = line["c2_fresh_cold"]["compute_frac_peak"]
            del tx, rx
            side("c4_shard", lambda: c4_shard(ctx, torch, args.steps, args.warmup, args.settle_s))
            side("c1_64B", lambda: c1_small_frames(ctx, torch))
            side("c1_64B_8M", lambda: c1_small_frames(ctx, torch, n=8 << 20))
            side("c2_1514B", lambda: c2_max_frame(ctx, torch))
            side("c3_imix", lambda: c3_imix(ctx, torch))
            side("c2_rooms", lambda: c2_rooms(ctx, torch))
            side("rows_8f", lambda: rows_8f(ctx, torch))
            side("pcie_inclusive", lambda: pcie_inclusive(gpucsum, torch))
            side("plugin_bursts", lambda: plugin_bursts(gpucsum))
            side("plugin_threads", plugin_threads)
            side("plugin_tx_async", plugin_tx_async)
            side("plugin_rx_async", plugin_rx_async)
            side("server_poll_cost", server_poll_cost)
    ctx.close()
    if rank == 0:
        extras = None
        if any(k not in compact_line(line) for k in line):
            # the full tables beside the line (never in it: the driver parses
            # ONE line, and round 5's 29 KB line was left unparsed)
            extras = EXTRAS_PATH
            try:
                with open(extras, "w") as f:
                    json.dump(line, f)
            except OSError as e:
                print(f"warning: extras not written: {e}", file=sys.stderr)
                extras = None
        print(json.dumps(compact_line(line, extras)), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
