"""C2 step, fused (gcs_step_fixed_dev: one launch) against split (TX fill
launch + RX verify launch), alternating blocks of 20 timed steps after a
settle, same batches (tools/, not product).  Prints one JSON object."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from mtcp_amd import gpucsum  # noqa: E402


def main():
    n = int(os.environ.get("SA_FRAMES", str(1 << 20)))
    L = 1500
    ctx = gpucsum.Context(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = torch.cuda.current_stream().cuda_stream
    tx, rx, stride, nbad = bench.make_batches(ctx, n, L, 0x6D746370, torch)
    v = torch.empty(n, dtype=torch.uint8, device="cuda")

    def split():
        ctx.compute_fixed(tx, stride, L, n, stream=stream)
        ctx.verify_fixed(rx, stride, L, n, v, stream=stream)

    def fused():
        ctx.step_fixed(tx, stride, L, n, rx, stride, L, n, v, stream=stream)

    def timed(fn, steps=20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3, e0.elapsed_time(e1) / steps

    t_end = time.perf_counter() + 1.0
    while time.perf_counter() < t_end:
        for _ in range(10):
            split()
            fused()
        torch.cuda.synchronize()
    out = {"frames": n, "split_ms": [], "fused_ms": [], "split_event_ms": [], "fused_event_ms": []}
    for _ in range(6):
        for name, fn in (("split", split), ("fused", fused)):
            w, e = timed(fn)
            out[name + "_ms"].append(round(w, 4))
            out[name + "_event_ms"].append(round(e, 4))
    assert int((v != 0).sum()) == nbad
    for k in ("split_ms", "fused_ms", "split_event_ms", "fused_event_ms"):
        out[k + "_median"] = round(float(np.median(out[k])), 4)
    out["fused_gpkt_per_s"] = round(2 * n / out["fused_ms_median"] / 1e6, 4)
    out["split_gpkt_per_s"] = round(2 * n / out["split_ms_median"] / 1e6, 4)
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
