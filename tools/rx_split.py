"""Where an RX burst's blocked time goes (tools/, not product).

gcs_verify_ptrs on 64 x 1500 B frames in 2 KiB rooms, the call the plugin
makes in recv_pkts for one batch per burst (GPUCSUM_RX_GROUP=0), through the
burst server, each burst's frames first written into the rooms as a NIC
would.  Per call (C clock_gettime, tools/libburst_timer.so) and, from the
counting grid (GCS_SERVER_COUNTERS=1, gcs_server_stats_get):

  post_to_done   the request posted -> its records seen by the host
  seen_wait      post -> the first serving block saw it (over the fastest)
  gpu_span       first block saw it -> last block's records stored
  after_gpu      records stored -> host done (plus the fastest post -> seen)
  acquire / frames / records   per serving block

so call - post_to_done is the host's own work around the request (find the
region, descriptors, verdicts out, the tcp_in.c:1237 side effect).

Environment: RXS_ROOMS=registered (default; read in place over PCIe) or
pageable (staged by the host into device memory over the BAR); RXS_BURSTS
(default 400); the library's GCS_SERVER_* knobs.  Prints one JSON object.
"""
import ctypes as C
import json
import os
import sys

import numpy as np

os.environ.setdefault("GCS_SERVER_COUNTERS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (one HIP runtime per process: torch first)
from mtcp_amd import gpucsum, synth  # noqa: E402
from oracle_lib import Oracle  # noqa: E402


class Stats(C.Structure):
    _fields_ = ([(k, C.c_uint64) for k in ("requests", "block_requests", "polls")] +
                [(k, C.c_double) for k in ("post_to_done_us", "gpu_span_us", "poll_us",
                                           "seen_poll_us", "acquire_us", "frames_us",
                                           "records_us", "release_us", "seen_skew_us",
                                           "block_serve_us", "cold_frac")] +
                [(k, C.c_uint64) for k in ("slow_polls_2us", "slow_polls_5us", "torn_polls")] +
                [("max_poll_us", C.c_double), ("late_us", C.c_double * 8),
                 ("seen_wait_us", C.c_double), ("after_gpu_us", C.c_double)])


def main():
    vp, u32 = C.c_void_p, C.c_uint32
    P = gpucsum.lib()
    P.gcs_server_stats_get.argtypes = [vp, C.POINTER(Stats)]
    T = C.CDLL(os.path.join(ROOT, "tools", "libburst_timer.so"))
    T.bt_run.argtypes = [vp, vp, vp, vp, u32, vp, vp, u32, vp]
    burst, L = 64, 1500
    bursts = int(os.environ.get("RXS_BURSTS", "400"))
    registered = os.environ.get("RXS_ROOMS", "registered") == "registered"
    n = burst * bursts
    src, stride = synth.fixed_frames(n, L, seed=0x5A)
    off = np.arange(n, dtype=np.uint64) * stride
    lens = np.full(n, L, dtype=np.uint16)
    Oracle().compute_batch(src, off, lens)
    synth.corrupt(src, off, lens, frac_log2=6, seed=0x5B)
    ref = Oracle().verify_batch(src.copy(), off, lens, flags=1)
    mem = np.zeros(burst * 2048 + 8192, np.uint8)
    base = (-mem.ctypes.data) % 4096
    rooms = mem[base:base + burst * 2048]
    ptrs = (vp * burst)(*[rooms.ctypes.data + 2048 * i for i in range(burst)])
    ln = np.full(burst, L, np.uint16)
    verdict = np.zeros(burst, np.uint8)
    t = np.zeros(bursts, np.float64)
    fn = C.cast(P.gcs_verify_ptrs, vp)
    wrong = 0
    if registered:
        gpucsum.check(P.gcs_host_register(vp(rooms.ctypes.data), rooms.nbytes), "register")
    try:
        with gpucsum.Context(0, max_frames=4096, max_bytes=8 << 20) as ctx:
            ctx.set_burst_server(True)
            for k in range(bursts):
                rv = rooms.reshape(burst, 2048)
                rv[:, :L] = src[k * burst * stride:(k + 1) * burst * stride].reshape(
                    burst, stride)[:, :L]
                gpucsum.check(T.bt_run(fn, ctx.h, ptrs, ln.ctypes.data, burst,
                                       verdict.ctypes.data, vp(1), 1, t[k:].ctypes.data),
                              "verify")
                wrong += int((verdict != ref[k * burst:(k + 1) * burst]).sum())
            st = Stats()
            gpucsum.check(P.gcs_server_stats_get(ctx.h, C.byref(st)), "stats")
    finally:
        if registered:
            gpucsum.check(P.gcs_host_unregister(vp(rooms.ctypes.data)), "unregister")
    tt = t[20:]
    out = {"rooms": "registered (in place)" if registered else "pageable (staged)",
           "config": {k: os.environ.get(k, "default") for k in
                      ("GCS_SERVER_ACQUIRE", "GCS_SERVER_COUNTERS", "GCS_SERVER_WAIT",
                       "GCS_DIRECT_STAGE")},
           "bursts": bursts, "wrong_verdicts": wrong,
           "call_us_median": round(float(np.median(tt)), 3),
           "call_us_p90": round(float(np.percentile(tt, 90)), 3)}
    for k in ("post_to_done_us", "seen_wait_us", "gpu_span_us", "after_gpu_us", "poll_us",
              "seen_poll_us", "acquire_us", "frames_us", "records_us", "block_serve_us",
              "cold_frac"):
        out[k] = round(getattr(st, k), 3)
    out["host_outside_request_us"] = round(out["call_us_median"] - out["post_to_done_us"], 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
