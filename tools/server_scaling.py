"""Burst-server scaling with the number of rings, phase by phase (tools/, not
product).  One configuration per process (the hub reads GCS_SERVER_MAILBOX /
GCS_SERVER_ACQUIRE / GCS_SERVER_COUNTERS once); every ring reports
gcs_server_stats' GPU-side phases from the grid's counters.

Two drivers (tests/plugin/mt_bursts.c):
  threads   one mTCP-like thread per ring, synchronous 64-frame IMIX fill +
            verify per iteration (as the plugin's default bursts), every 16th
            burst checked against the oracle;
  rings     T threads each posting async bursts on R rings, then waiting:
            T x R hot rings with only T CPUs busy (no oversubscription).
Prints one JSON object."""
import ctypes as C
import json
import os
import sys

# SS_PROF=1: the grid build with phase counters (GPU serving time and its
# phases); 0: the shipped plain build (host-side figures only)
os.environ["GCS_SERVER_COUNTERS"] = "1" if os.environ.get("SS_PROF", "1") == "1" else "0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mtcp_amd import gpucsum  # noqa: E402

gpucsum.lib()
M = C.CDLL(os.path.join(ROOT, "tests", "plugin", "libmt_bursts.so"))
M.mt_bursts.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint64),
                        C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
M.mt_rings.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint64),
                       C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
M.mt_last_cpu_frac.restype = C.c_double
M.mt_last_server_stats.argtypes = [C.POINTER(C.c_double), C.c_int]
KEYS = ["requests", "post_to_done_us", "gpu_span_us", "poll_us", "seen_poll_us", "acquire_us",
        "frames_us", "records_us", "release_us", "polls_per_block_request", "seen_skew_us",
        "block_serve_us", "cold_frac", "slow_polls_2us", "slow_polls_5us", "torn_polls",
        "max_poll_us"] + [f"late_us_b{b}" for b in range(8)] + ["seen_wait_us", "after_gpu_us"]


def server_stats():
    a = (C.c_double * len(KEYS))()
    M.mt_last_server_stats(a, len(KEYS))
    return {k: round(a[i], 3) for i, k in enumerate(KEYS)}


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


def main():
    os.environ["MT_CHECK_EVERY"] = os.environ.get("MT_CHECK_EVERY", "16")
    out = {"config": {k: os.environ.get(k, "default") for k in
                      ("GCS_SERVER_MAILBOX", "GCS_SERVER_ACQUIRE", "GCS_SERVER_COUNTERS",
                       "GCS_DIRECT_STAGE", "GCS_SERVER_HOT_NAPS", "GCS_SERVER_HOT_US",
                       "GCS_SERVER_WAIT", "GCS_SERVER_SPIN_US", "MT_PIN")},
           "cpus": cpu_quota(),
           "cpu_frac": "thread CPU time / wall time inside the calls (below 1: descheduled)"}
    iters = int(os.environ.get("SS_ITERS", "600"))
    for threads in [int(x) for x in os.environ.get("SS_THREADS", "1,4,8,12,16").split(",") if x]:
        mis, fr, us = C.c_uint64(), C.c_uint64(), C.c_double()
        rc = M.mt_bursts(threads, iters, 1, C.byref(mis), C.byref(fr), C.byref(us))
        assert rc == 0 and mis.value == 0, (rc, mis.value)
        out[f"threads_{threads}"] = dict(us_per_call=round(us.value, 3),
                                         cpu_frac=round(M.mt_last_cpu_frac(), 3), **server_stats())
        print(f"threads {threads}: {out[f'threads_{threads}']}", file=sys.stderr, flush=True)
    for spec in os.environ.get("SS_RINGS", "4x1,4x2,4x4,4x6").split(","):
        if not spec:
            continue
        t, r = (int(x) for x in spec.split("x"))
        mis, fr, us = C.c_uint64(), C.c_uint64(), C.c_double()
        rc = M.mt_rings(t, r, iters, C.byref(mis), C.byref(fr), C.byref(us))
        assert rc == 0 and mis.value == 0, (rc, mis.value)
        out[f"rings_{t}x{r}"] = dict(us_per_round=round(us.value, 3),
                                     cpu_frac=round(M.mt_last_cpu_frac(), 3), **server_stats())
        print(f"rings {t}x{r}: {out[f'rings_{t}x{r}']}", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
