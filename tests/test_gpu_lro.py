"""Software LRO on the GPU (gcs_gro_dev) against the oracle
(ref_gro_batch): run heads, output offsets / lengths and every output frame
byte for byte; merged frames pass the RX verify."""
import numpy as np
import pytest

from mtcp_amd import gpucsum, synth
from oracle_lib import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (no CPU fallback exists)")
    return torch


@pytest.fixture(scope="module")
def ctx(torch_dev):
    c = gpucsum.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def O():
    return Oracle()


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.cpu().numpy()


def run_gro(t, ctx, buf, off, lens, vd, window, max_len, out_bytes=None, in_bytes=None):
    n = len(off)
    ob = buf.nbytes if out_bytes is None else out_bytes
    out = t.zeros(ob, dtype=t.uint8, device="cuda")
    oo = t.zeros(n, dtype=t.int64, device="cuda")
    ol = t.zeros(n, dtype=t.int16, device="cuda")
    hd = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.gro(dev(t, buf), dev(t, off.view(np.int64)), dev(t, lens.view(np.int16)), dev(t, vd), n,
            window, max_len, out, oo, ol, hd, in_bytes=in_bytes)
    ctx.sync()
    return (host(out), host(oo).view(np.uint64), host(ol).view(np.uint16),
            host(hd).view(np.uint32))


def compare(buf, off, lens, gpu, ref):
    out, oo, ol, hd = gpu
    rout, roo, rol, rhd = ref
    np.testing.assert_array_equal(hd, rhd)
    np.testing.assert_array_equal(oo, roo)
    np.testing.assert_array_equal(ol, rol)
    heads = np.nonzero(hd == np.arange(len(off)))[0]
    for h in heads:
        a, b = int(oo[h]), int(oo[h]) + int(ol[h])
        np.testing.assert_array_equal(out[a:min(b, len(out))], rout[a:min(b, len(rout))])
    return heads


def verdicts(t, ctx, buf, off, lens):
    n = len(off)
    v = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.verify(dev(t, buf), dev(t, off.view(np.int64)), dev(t, lens.view(np.int16)), n, v)
    ctx.sync()
    return host(v)


@pytest.mark.parametrize("window,max_len,run_mean", [(64, 16384, 6.0), (256, 65535, 50.0),
                                                     (1, 16384, 6.0), (7, 3000, 6.0),
                                                     (256, 16384, 3.0), (65, 16384, 6.0),
                                                     (100, 3000, 20.0), (200, 16384, 40.0),
                                                     (256, 3000, 20.0)])
def test_gro_streams_vs_oracle(torch_dev, ctx, O, window, max_len, run_mean):
    t = torch_dev
    n = 20000
    buf, off, lens = synth.tcp_streams(n, run_mean=run_mean, seed=window + max_len)
    O.compute_batch(buf, off, lens)
    synth.corrupt(buf, off, lens, frac_log2=6, seed=3)       # a few bad frames: never merged
    vd = verdicts(t, ctx, buf, off, lens)
    np.testing.assert_array_equal(vd, O.verify_batch(buf.copy(), off, lens))
    gpu = run_gro(t, ctx, buf, off, lens, vd, window, max_len)
    ref = O.gro_batch(buf, off, lens, vd, window, max_len)
    heads = compare(buf, off, lens, gpu, ref)
    if window > 1:
        assert len(heads) < n * 0.8
    # every merged frame passes the RX verify
    out, oo, ol, hd = gpu
    merged = np.array([h for h in heads if (hd == h).sum() > 1], dtype=np.int64)
    if len(merged):
        v = O.verify_batch(out.copy(), oo[merged], ol[merged])
        assert (v == 0).all()


@pytest.mark.parametrize("window", [64, 200, 256])
def test_gro_mixed_traffic_and_bad_descriptors(torch_dev, ctx, O, window):
    """Streams interleaved with IMIX frames, ICMP, bad descriptors and a
    cut-short output buffer; windows of 64 (wave 0 plans) and of more frames
    (the block plans: chains and segments across waves)."""
    t = torch_dev
    rng = np.random.default_rng(9)
    sb, so, sl = synth.tcp_streams(3000, seed=10)
    ib, io, il = synth.packed_frames(synth.imix_lengths(1000, seed=11), seed=12)
    # interleave: frames of both sets, re-packed
    order = np.argsort(rng.random(4000), kind="stable")
    frames = [(sb, so[k], sl[k]) for k in range(3000)] + [(ib, io[k], il[k]) for k in range(1000)]
    frames = [frames[k] for k in order]
    lens = np.array([L for _, _, L in frames], dtype=np.uint16)
    off, total = synth.packed_offsets(lens)
    buf = np.zeros(total + 64, dtype=np.uint8)
    for (b, o, L), oo in zip(frames, off):
        buf[int(oo):int(oo) + int(L)] = b[int(o):int(o) + int(L)]
    O.compute_batch(buf, off, lens)
    for k in rng.choice(4000, 100, replace=False):
        buf[int(off[k]) + 23] = 1                             # ICMP: not ACCEPT
    off = off.copy()
    off[5] += 8                                               # misaligned descriptor
    off[2 * window] += 8                                      # ... first of its window: the
    vd = verdicts(t, ctx, buf, off, lens)                     # window's output base moves too
    for out_bytes in (None, buf.nbytes // 2 + 3):
        gpu = run_gro(t, ctx, buf, off, lens, vd, window, 16384, out_bytes=out_bytes)
        ref = O.gro_batch(buf, off, lens, vd, window, 16384, out_bytes=out_bytes)
        compare(buf, off, lens, gpu, ref)
        assert gpu[2][5] == 0 and gpu[2][2 * window] == 0


def test_gro_rejects_bad_arguments(torch_dev, ctx):
    t = torch_dev
    z = t.zeros(64, dtype=t.uint8, device="cuda")
    o = t.zeros(1, dtype=t.int64, device="cuda")
    ln = t.full((1,), 64, dtype=t.int16, device="cuda")
    h = t.zeros(1, dtype=t.int32, device="cuda")
    for window, max_len in ((0, 100), (257, 100), (64, 70000)):
        with pytest.raises(gpucsum.GcsError):
            ctx.gro(z, o, ln, z, 1, window, max_len, z, o, ln, h)
