"""The burst server next to a device-resident batch kernel (tools/,
not product): software LRO (gcs_gro_dev, 1M x 1500 B, windows of 64, ~52 KB
of LDS per 1,024-thread block) timed alone and while SL_THREADS mTCP-like
threads push 64-frame bursts through the server grid (tests/plugin/
mt_bursts.c), whose blocks each reserve GCS_SERVER_LDS_KB (default 96) KiB of
LDS; and the bursts' per-call time alone and beside the LRO launches.
Prints one JSON object."""
import ctypes as C
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from mtcp_amd import gpucsum, synth  # noqa: E402

os.environ.setdefault("MT_CHECK_EVERY", "16")
gpucsum.lib()
M = C.CDLL(os.path.join(ROOT, "tests", "plugin", "libmt_bursts.so"))
M.mt_bursts.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint64),
                        C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
M.mt_last_cpu_frac.restype = C.c_double


def bursts(threads, iters):
    mis, fr, us = C.c_uint64(), C.c_uint64(), C.c_double()
    rc = M.mt_bursts(threads, iters, 1, C.byref(mis), C.byref(fr), C.byref(us))
    assert rc == 0 and mis.value == 0, (rc, mis.value)
    return us.value


def main():
    threads = int(os.environ.get("SL_THREADS", "8"))
    n, L = 1 << 20, 1500
    ctx = gpucsum.Context(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = torch.cuda.current_stream().cuda_stream
    sb, stride = synth.tcp_streams_device(n, L)
    off = torch.arange(n, device="cuda", dtype=torch.int64) * stride
    lens = torch.full((n,), L, dtype=torch.int16, device="cuda")
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.compute(sb, off, lens, n, stream=stream)
    ctx.verify(sb, off, lens, n, v, stream=stream)
    o = torch.empty_like(sb)
    oo = torch.empty(n, dtype=torch.int64, device="cuda")
    ol = torch.empty(n, dtype=torch.int16, device="cuda")
    hd = torch.empty(n, dtype=torch.int32, device="cuda")

    def lro_ms(reps=20):
        for _ in range(3):
            ctx.gro(sb, off, lens, v, n, 64, 16384, o, oo, ol, hd, stream=stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            ctx.gro(sb, off, lens, v, n, 64, 16384, o, oo, ol, hd, stream=stream)
        e1.record()
        torch.cuda.synchronize()
        assert int((ol != 0).sum()) == n // 8
        return e0.elapsed_time(e1) / reps

    out = {"config": {k: os.environ.get(k, "default") for k in
                      ("GCS_SERVER_LDS_KB", "GCS_SERVER_LDS_GROUPS", "SL_THREADS")},
           "workload": f"LRO 1M x 1500 B windows of 64 (20 launches) beside {threads} threads of "
                       "64-frame IMIX fill+verify bursts through the server"}
    out["lro_ms_alone"] = [round(lro_ms(), 4) for _ in range(3)]
    out["burst_us_alone"] = round(bursts(threads, 2000), 3)
    res = {}
    th = threading.Thread(target=lambda: res.update(us=bursts(threads, 10000)))
    th.start()
    time.sleep(0.005)                   # the grid is up and its rings hot
    busy = []
    while th.is_alive():                # LRO launches for as long as the bursts run
        busy.append(round(lro_ms(10), 4))
    th.join()
    out["lro_ms_beside_bursts"] = busy
    out["burst_us_beside_lro"] = round(res["us"], 3)
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
