"""Burst latency with several mTCP-like threads per GPU (tests/plugin/mt_bursts.c),
as the plugin runs them (GPU_MAX_HW_QUEUES=16 when run through bench.py).
Prints one JSON object (tools/, not product)."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mtcp_amd import gpucsum  # noqa: E402

gpucsum.lib()
M = C.CDLL(os.path.join(ROOT, "tests", "plugin", "libmt_bursts.so"))
M.mt_bursts.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint64),
                        C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
M.mt_last_cpu_frac.restype = C.c_double


def cpu_quota():
    """CPUs this process may use: affinity, and the cgroup v2 quota if any."""
    q = None
    try:
        a, b = open("/sys/fs/cgroup/cpu.max").read().split()
        if a != "max":
            q = int(a) / int(b)
    except (OSError, ValueError):
        pass
    return {"affinity": len(os.sched_getaffinity(0)), "cgroup_quota": q}


out = {"workload": "threads each with its own context on GPU 0, 64-frame IMIX bursts "
                   "(fill + verify), every frame checked against the oracle; mean us per call "
                   "inside the gcs calls",
       "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "default (4)"),
       "cpus": cpu_quota(),
       "cpu_frac": "thread CPU time / wall time inside the calls (below 1: descheduled)"}
for threads in [int(x) for x in os.environ.get("MTP_THREADS", "1,4,8,12,16,24").split(",")]:
    for server in (1, 0):
        mis, fr, us = C.c_uint64(), C.c_uint64(), C.c_double()
        rc = M.mt_bursts(threads, 300, server, C.byref(mis), C.byref(fr), C.byref(us))
        assert rc == 0 and mis.value == 0, (rc, mis.value)
        out[f"{threads}_threads_{'server' if server else 'launch'}_us"] = us.value
        out[f"{threads}_threads_{'server' if server else 'launch'}_cpu_frac"] = \
            M.mt_last_cpu_frac()
# the same with new frames and the oracle check on every 16th burst only: the
# threads' own CPU work no longer crowds the job's cores (cgroup quota above)
os.environ["MT_CHECK_EVERY"] = "16"
for threads in [int(x) for x in os.environ.get("MTP_LIGHT_THREADS", "1,8,12,16,24").split(",") if x]:
    mis, fr, us = C.c_uint64(), C.c_uint64(), C.c_double()
    rc = M.mt_bursts(threads, 600, 1, C.byref(mis), C.byref(fr), C.byref(us))
    assert rc == 0 and mis.value == 0, (rc, mis.value)
    out[f"{threads}_threads_server_light_us"] = us.value
    out[f"{threads}_threads_server_light_cpu_frac"] = M.mt_last_cpu_frac()
del os.environ["MT_CHECK_EVERY"]
print(json.dumps(out))
