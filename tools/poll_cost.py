"""What idle burst-server grids cost the PCIe link (tools/, not product).

K helper threads each own a context with the burst server on and post a
one-frame burst every ~200 us, so their grids stay resident and poll their
mailboxes in host memory between bursts (as the grids of K mTCP threads per
GPU do).  Meanwhile the main thread runs the PCIe-inclusive verify of
bench.py (1M x 1500 B pinned host frames: H2D copies, kernel, D2H verdicts)
and reports its rate for K = 0, 8, 12 (PC_KS).  PC_HELPER_SERVER=0 runs the
helpers without the burst server (a launch per burst): the control that
separates what idle grids cost from what the helpers' bursts cost.  Prints
one JSON object."""
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process: torch first)
from mtcp_amd import gpucsum, synth  # noqa: E402

L_ = gpucsum.lib()
N, FL = int(os.environ.get("PC_FRAMES", str(1 << 20))), 1500
src, stride = synth.fixed_frames(N, FL, seed=77)
off = np.arange(N, dtype=np.uint64) * stride
lens = np.full(N, FL, dtype=np.uint16)
pinned = gpucsum.PinnedBuffer(src.nbytes)
pinned.array[:] = src
HELPER_SERVER = os.environ.get("PC_HELPER_SERVER", "1") != "0"
KS = [int(k) for k in os.environ.get("PC_KS", "0,8,12,0").split(",")]


def helper(stop, stats):
    one, ostride = synth.fixed_frames(1, 1500, seed=5)
    with gpucsum.Context(0, max_frames=64, max_bytes=1 << 20) as c:
        c.set_burst_server(HELPER_SERVER)
        v = np.zeros(1, np.uint8)
        ptrs = (C.c_void_p * 1)(one.ctypes.data)
        ln = np.full(1, 1500, np.uint16)
        k = 0
        while not stop.is_set():
            gpucsum.check(L_.gcs_verify_ptrs(c.h, ptrs, ln.ctypes.data, 1, v.ctypes.data, 0))
            k += 1
            time.sleep(200e-6)
        stats.append(k)


out = {"workload": f"verify of {N} x {FL} B pinned host frames (gcs_verify: H2D, kernel, D2H) "
                   "while K other contexts' burst-server grids poll between 1-frame bursts "
                   "every ~200 us",
       "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "default (4)"),
       "helper_server": HELPER_SERVER,
       "GCS_SERVER_HOT_US": os.environ.get("GCS_SERVER_HOT_US", "default (20)")}
with gpucsum.Context(0, max_frames=1 << 16, max_bytes=96 << 20) as c:
    c.compute_host(pinned.array, off, lens)            # valid checks: every frame accepted
    for K in KS:
        stop, stats = threading.Event(), []
        th = [threading.Thread(target=helper, args=(stop, stats)) for _ in range(K)]
        for t in th:
            t.start()
        time.sleep(0.3)
        c.verify_host(pinned.array, off, lens)
        reps, t0 = 5, time.perf_counter()
        for _ in range(reps):
            codes = c.verify_host(pinned.array, off, lens)
        dt = (time.perf_counter() - t0) / reps
        stop.set()
        for t in th:
            t.join()
        assert int((codes != 0).sum()) == 0
        key = f"K{K}"
        while key in out:
            key += "_again"
        out[key] = {"gib_per_s": N * FL / dt / 2**30, "gb_per_s_h2d": N * stride / dt / 1e9,
                    "helper_bursts": int(sum(stats))}
pinned.free()
print(json.dumps(out))
