"""Randomized parity stress for the round-3 stream kernels (tools/, not part of
the suite): k_desc_stream (descriptor verify / fill) and k_gro FLAT (LRO)
against the oracle over many seeds, packings, header mixes, window sizes and
max_len cuts.  Prints one JSON line with the case counts; raises on the first
mismatch.  Run on a GPU box: python tools/stress_stream.py [cases]."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from mtcp_amd import gpucsum, synth  # noqa: E402
from oracle_lib import Oracle  # noqa: E402
from test_gpu_parity import stream_case_frames  # noqa: E402


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def desc_case(ctx, O, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 256 * 12))
    align = int(rng.choice([16, 64]))
    jumbo = float(rng.choice([0.0, 0.0, 0.01, 0.05]))
    buf, off, lens = stream_case_frames(n, align, seed=seed, jumbo=jumbo)
    off = off.copy()
    if n > 10 and rng.random() < 0.3:                 # a misordered pair somewhere
        k = int(rng.integers(0, n - 1))
        off[k], off[k + 1] = off[k + 1], off[k]
        lens[k], lens[k + 1] = lens[k + 1], lens[k]
    doff, dlen = dev(off.view(np.int64)), dev(lens.view(np.int16))
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens)
    d = dev(buf)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cs = torch.zeros(n, dtype=torch.int32, device="cuda")
    ctx.compute(d, doff, dlen, n, st, cs)
    ctx.sync()
    assert np.array_equal(st.cpu().numpy(), rst), f"desc fill status, seed {seed}"
    assert np.array_equal(cs.cpu().numpy().view(np.uint32), rcs), f"desc fill csums, seed {seed}"
    assert np.array_equal(d.cpu().numpy(), ref), f"desc fill bytes, seed {seed}"
    synth.corrupt(ref, off, np.maximum(lens, 15), frac_log2=3, seed=seed)
    flags = int(rng.integers(0, 2))
    d = dev(ref)
    v = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    ctx.verify(d, doff, dlen, n, v, flags=flags)
    ctx.sync()
    exp = ref.copy()
    rv = O.verify_batch(exp, off, lens, flags=flags)
    assert np.array_equal(v.cpu().numpy(), rv), f"desc verify, seed {seed}"
    assert np.array_equal(d.cpu().numpy(), exp), f"desc verify side effect, seed {seed}"
    return n


def gro_case(ctx, O, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 6000))
    window = int(rng.choice([1, 3, 7, 16, 33, 64, 64, 64, 65, 100, 200, 256, 256]))
    max_len = int(rng.choice([200, 3000, 9000, 16384, 65535]))
    run_mean = float(rng.choice([1.5, 3.0, 6.0, 20.0]))
    buf, off, lens = synth.tcp_streams(n, run_mean=run_mean, seed=seed)
    O.compute_batch(buf, off, lens)
    synth.corrupt(buf, off, lens, frac_log2=5, seed=seed + 1)
    vd = O.verify_batch(buf.copy(), off, lens)
    out_bytes = buf.nbytes if rng.random() < 0.8 else int(buf.nbytes * rng.uniform(0.3, 1.0))
    out = torch.zeros(out_bytes, dtype=torch.uint8, device="cuda")
    oo = torch.zeros(n, dtype=torch.int64, device="cuda")
    ol = torch.zeros(n, dtype=torch.int16, device="cuda")
    hd = torch.zeros(n, dtype=torch.int32, device="cuda")
    ctx.gro(dev(buf), dev(off.view(np.int64)), dev(lens.view(np.int16)), dev(vd), n, window,
            max_len, out, oo, ol, hd)
    ctx.sync()
    rout, roo, rol, rhd = O.gro_batch(buf, off, lens, vd, window, max_len, out_bytes=out_bytes)
    g_out, g_oo = out.cpu().numpy(), oo.cpu().numpy().view(np.uint64)
    g_ol, g_hd = ol.cpu().numpy().view(np.uint16), hd.cpu().numpy().view(np.uint32)
    assert np.array_equal(g_hd, rhd) and np.array_equal(g_oo, roo) and np.array_equal(g_ol, rol), \
        f"gro tables, seed {seed} window {window} max_len {max_len}"
    for h in np.nonzero(g_hd == np.arange(n))[0]:
        a, b = int(g_oo[h]), int(g_oo[h]) + int(g_ol[h])
        assert np.array_equal(g_out[a:min(b, len(g_out))], rout[a:min(b, len(rout))]), \
            f"gro bytes, seed {seed} head {h}"
    return n


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    O = Oracle()
    frames = {"desc": 0, "gro": 0}
    with gpucsum.Context(0, max_frames=1 << 16, max_bytes=64 << 20) as ctx:
        for s in range(cases):
            frames["desc"] += desc_case(ctx, O, 1000 + s)
            frames["gro"] += gro_case(ctx, O, 2000 + s)
            print(f"case {s}: ok", flush=True, file=sys.stderr)
    print(json.dumps({"cases": cases, "frames": frames, "result": "all equal"}))


if __name__ == "__main__":
    main()
