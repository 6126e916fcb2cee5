"""SURVEY §8f rows 2-3 on the GPU: the ICMP fold (ICMPChecksum, icmp.c:18-42,
inside the batched verify / fill) and RSS steering (GetRSSHash /
GetRSSCPUCore, rss.c:44-115, fused into the RX verify), through the C ABI,
bit-exact against the reference's golden vectors and the oracle.
"""
import hashlib
import os

import numpy as np
import pytest

from mtcp_amd import gpucsum, synth
from oracle_lib import Oracle

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
K = gpucsum.K
VF_ICMP, CF_ICMP = K["GCS_VF_ICMP"], K["GCS_CF_ICMP"]


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (no CPU fallback exists)")
    return torch


@pytest.fixture(scope="module")
def ctx(torch_dev):
    c = gpucsum.Context(0, max_frames=1 << 16, max_bytes=64 << 20)
    yield c
    c.close()


@pytest.fixture(scope="module")
def O():
    return Oracle()


def load(name):
    with np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.cpu().numpy()


def zeros(t, n, dtype):
    return t.zeros(n, dtype=dtype, device="cuda")


# ---------------------------------------------------------------------------
# golden vectors from the reference (icmp.c / rss.c compiled in place)

def test_golden_icmp_fn(torch_dev, ctx):
    t = torch_dev
    d = load("icmp_fn")
    n = len(d["off"])
    out = zeros(t, n, t.int16)
    ctx.icmp_checksum(dev(t, d["buf"]), dev(t, d["off"].view(np.int64)),
                      dev(t, d["len"].view(np.int16)), n, out)
    ctx.sync()
    np.testing.assert_array_equal(host(out).view(np.uint16), d["expect"])


def test_golden_rss(torch_dev, ctx):
    t = torch_dev
    d = load("rss")
    n = len(d["sip"])
    args = [dev(t, d[k].view(np.int32 if d[k].dtype == np.uint32 else np.int16))
            for k in ("sip", "dip", "sp", "dp")]
    for a, nq in enumerate(d["nq"]):
        for e in (0, 1):
            ctx.set_rss(None, int(nq), e)
            h = zeros(t, n, t.int32)
            q = zeros(t, n, t.int16)
            ctx.rss(*args, n, h, q)
            ctx.sync()
            np.testing.assert_array_equal(host(h).view(np.uint32), d["hash"])
            np.testing.assert_array_equal(host(q).view(np.uint16), d["core"][a, e])
    ctx.set_rss(None, 1, 0)


def test_golden_frames_l4(torch_dev, ctx):
    t = torch_dev
    d = load("frames_l4")
    n = len(d["off"])
    doff, dlen = dev(t, d["off"].view(np.int64)), dev(t, d["len"].view(np.int16))
    for flags, key in ((VF_ICMP, "rx"), (0, "rx_noflag")):
        v = zeros(t, n, t.uint8)
        ctx.verify(dev(t, d["buf"]), doff, dlen, n, v, flags=flags)
        ctx.sync()
        np.testing.assert_array_equal(host(v), d[key])
    for k in range(2):
        ctx.set_rss(None, int(d["rss_nq"][k]), int(d["rss_endian"][k]))
        v = zeros(t, n, t.uint8)
        h = zeros(t, n, t.int32)
        q = zeros(t, n, t.int16)
        ctx.classify(dev(t, d["buf"]), doff, dlen, n, v, h, q, flags=VF_ICMP)
        ctx.sync()
        vd = host(v)
        np.testing.assert_array_equal(vd, d["rx"])
        acc = vd == 0
        hh, qq = host(h).view(np.uint32), host(q).view(np.uint16)
        np.testing.assert_array_equal(hh[acc], d["rss_hash"][acc])
        np.testing.assert_array_equal(qq[acc], d["rss_core"][k][acc])
        assert (qq[~acc] == 0xFFFF).all() and (hh[~acc] == 0).all()
    ctx.set_rss(None, 1, 0)
    buf = dev(t, d["tx"])
    st = zeros(t, n, t.uint8)
    cs = zeros(t, n, t.int32)
    ctx.compute(buf, doff, dlen, n, st, cs, flags=CF_ICMP)
    ctx.sync()
    np.testing.assert_array_equal(host(st), d["tx_status"])
    np.testing.assert_array_equal(host(cs).view(np.uint32), d["tx_csums"])
    assert hashlib.sha256(host(buf).tobytes()).digest() == d["tx_filled_sha256"].tobytes()


# ---------------------------------------------------------------------------
# fixed-stride kernels, every dispatch class: TCP + ICMP mixes

FIXED_LENS = [42, 43, 51, 54, 60, 64, 100, 333, 576, 1024, 1500, 2001, 4000, 9000]


def mixed_fixed(n, L, seed):
    """TCP frames (>= 54 B) with every third frame turned into ICMP, or ICMP
    frames only below 54 B."""
    if L < 54:
        return synth.icmp_fixed_frames(n, L, seed=seed)
    buf, stride = synth.fixed_frames(n, L, seed=seed)
    off = np.arange(n, dtype=np.uint64) * stride
    synth.to_icmp(buf, off, np.full(n, L), np.arange(0, n, 3))
    return buf, stride


@pytest.mark.parametrize("frame_len", FIXED_LENS)
def test_fixed_icmp_fill_then_verify(torch_dev, ctx, O, frame_len):
    t = torch_dev
    n = 3000 if frame_len < 4000 else 600
    buf, stride = mixed_fixed(n, frame_len, seed=frame_len + 7)
    off = np.arange(n, dtype=np.uint64) * stride
    lens = np.full(n, frame_len, dtype=np.uint16)
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens, flags=2)
    d = dev(t, buf)
    st = zeros(t, n, t.uint8)
    cs = zeros(t, n, t.int32)
    ctx.compute_fixed(d, stride, frame_len, n, st, cs, flags=CF_ICMP)
    ctx.sync()
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)
    assert K["GCS_TX_ICMP_OK"] in set(rst.tolist())
    bad = synth.corrupt(ref, off, lens, frac_log2=3, seed=frame_len + 8)
    for flags in (VF_ICMP, VF_ICMP | 1, 0):
        d = dev(t, ref)
        v = zeros(t, n, t.uint8)
        ctx.verify_fixed(d, stride, frame_len, n, v, flags=flags)
        ctx.sync()
        r = ref.copy()
        rv = O.verify_batch(r, off, lens, flags=flags)
        np.testing.assert_array_equal(host(v), rv)
        np.testing.assert_array_equal(host(d), r)
    good = np.delete(np.arange(n), bad)
    rv = O.verify_batch(ref.copy(), off, lens, flags=VF_ICMP)
    assert set(rv[good].tolist()) <= {K["GCS_V_ACCEPT"], K["GCS_V_ICMP_OK"]}


@pytest.mark.parametrize("frame_len", [54, 60, 64, 100, 576, 1500, 4000])
@pytest.mark.parametrize("nq,endian,keyed", [(16, 0, False), (6, 1, False), (10, 1, True),
                                             (1, 0, True)])
def test_fixed_classify(torch_dev, ctx, O, frame_len, nq, endian, keyed):
    t = torch_dev
    n = 4000 if frame_len < 4000 else 800
    rng = np.random.default_rng(frame_len * 31 + nq)
    key = bytes(rng.integers(0, 256, 40, dtype=np.uint8)) if keyed else None
    buf, stride = mixed_fixed(n, frame_len, seed=frame_len + 99)
    off = np.arange(n, dtype=np.uint64) * stride
    lens = np.full(n, frame_len, dtype=np.uint16)
    O.compute_batch(buf, off, lens, flags=2)
    synth.corrupt(buf, off, lens, frac_log2=4, seed=nq)
    ctx.set_rss(key, nq, endian)
    try:
        rvd, rh, rq = O.classify_fixed(buf.copy(), stride, frame_len, n, nq, endian, key=key,
                                       flags=VF_ICMP)
        d = dev(t, buf)
        v = zeros(t, n, t.uint8)
        h = zeros(t, n, t.int32)
        q = zeros(t, n, t.int16)
        ctx.classify_fixed(d, stride, frame_len, n, v, h, q, flags=VF_ICMP)
        ctx.sync()
        np.testing.assert_array_equal(host(v), rvd)
        np.testing.assert_array_equal(host(h).view(np.uint32), rh)
        np.testing.assert_array_equal(host(q).view(np.uint16), rq)
        assert (rvd == 0).sum() > n // 3
        if nq > 1:
            assert len(np.unique(rq[rvd == 0])) > 1
        # queue only, no hash array
        q2 = zeros(t, n, t.int16)
        ctx.classify_fixed(d, stride, frame_len, n, v, None, q2)
        ctx.sync()
        _, _, rq0 = O.classify_fixed(buf.copy(), stride, frame_len, n, nq, endian, key=key)
        np.testing.assert_array_equal(host(q2).view(np.uint16), rq0)
    finally:
        ctx.set_rss(None, 1, 0)


# ---------------------------------------------------------------------------
# descriptor kernel (IMIX, fuzz) and the host entry points

def test_imix_icmp_and_classify(torch_dev, ctx, O):
    t = torch_dev
    n = 100_000
    lens = synth.imix_lengths(n, seed=21)
    buf, off, lens = synth.packed_frames(lens, seed=22)
    synth.to_icmp(buf, off, lens, np.arange(1, n, 5))
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens, flags=2)
    d = dev(t, buf)
    doff, dlen = dev(t, off.view(np.int64)), dev(t, lens.view(np.int16))
    st = zeros(t, n, t.uint8)
    cs = zeros(t, n, t.int32)
    ctx.compute(d, doff, dlen, n, st, cs, flags=CF_ICMP)
    ctx.sync()
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)
    synth.corrupt(ref, off, lens, frac_log2=5, seed=23)
    ctx.set_rss(None, 8, 0)
    try:
        rvd, rh, rq = O.classify_batch(ref.copy(), off, lens, 8, 0, flags=VF_ICMP)
        d = dev(t, ref)
        v = zeros(t, n, t.uint8)
        h = zeros(t, n, t.int32)
        q = zeros(t, n, t.int16)
        ctx.classify(d, doff, dlen, n, v, h, q, flags=VF_ICMP)
        ctx.sync()
        np.testing.assert_array_equal(host(v), rvd)
        np.testing.assert_array_equal(host(h).view(np.uint32), rh)
        np.testing.assert_array_equal(host(q).view(np.uint16), rq)
        # the host-memory entry point gives the same
        hv, hh, hq = ctx.classify_host(ref, off, lens, flags=VF_ICMP)
        np.testing.assert_array_equal(hv, rvd)
        np.testing.assert_array_equal(hh, rh)
        np.testing.assert_array_equal(hq, rq)
    finally:
        ctx.set_rss(None, 1, 0)


def test_fuzz_icmp_vs_oracle(torch_dev, ctx, O):
    """Random headers with protocol 1 or 6 and arbitrary lengths: ICMP verdicts,
    ICMP fills and the steering of ACCEPT frames all match the oracle."""
    from test_gpu_parity import fuzz_frames
    t = torch_dev
    n = 20000
    buf, off, lens = fuzz_frames(n, seed=41)
    rng = np.random.default_rng(42)
    for i in np.nonzero(rng.random(n) < 0.4)[0]:
        o = int(off[i])
        if lens[i] > 23:
            buf[o + 23] = 1
    tmp = buf.copy()
    O.compute_batch(tmp, off, lens, flags=2)
    sel = rng.random(n) < 0.5
    for i in np.nonzero(sel)[0]:
        o, L = int(off[i]), int(lens[i])
        buf[o:o + L] = tmp[o:o + L]
    d = dev(t, buf)
    doff, dlen = dev(t, off.view(np.int64)), dev(t, lens.view(np.int16))
    v = zeros(t, n, t.uint8)
    ctx.verify(d, doff, dlen, n, v, flags=VF_ICMP | 1)
    ctx.sync()
    ref = buf.copy()
    rv = O.verify_batch(ref, off, lens, flags=VF_ICMP | 1)
    np.testing.assert_array_equal(host(v), rv)
    np.testing.assert_array_equal(host(d), ref)
    assert {K["GCS_V_ICMP_OK"], K["GCS_V_ICMP_BADCSUM"]} <= set(rv.tolist())
    d = dev(t, buf)
    st = zeros(t, n, t.uint8)
    cs = zeros(t, n, t.int32)
    ctx.compute(d, doff, dlen, n, st, cs, flags=CF_ICMP)
    ctx.sync()
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens, flags=2)
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)
    assert {K["GCS_TX_ICMP_OK"], K["GCS_TX_BAD_ICMPLEN"]} <= set(rst.tolist())


def test_rss_custom_key_elementwise(torch_dev, ctx, O):
    t = torch_dev
    rng = np.random.default_rng(5)
    n = 50000
    key = bytes(rng.integers(0, 256, 40, dtype=np.uint8))
    sip = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    dip = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    sp = rng.integers(0, 1 << 16, n).astype(np.uint16)
    dp = rng.integers(0, 1 << 16, n).astype(np.uint16)
    ctx.set_rss(key, 12, 1)
    try:
        h = zeros(t, n, t.int32)
        q = zeros(t, n, t.int16)
        ctx.rss(dev(t, sip.view(np.int32)), dev(t, dip.view(np.int32)), dev(t, sp.view(np.int16)),
                dev(t, dp.view(np.int16)), n, h, q)
        ctx.sync()
        hh, qq = host(h).view(np.uint32), host(q).view(np.uint16)
        for i in range(0, n, 97):
            assert hh[i] == O.rss_hash(int(sip[i]), int(dip[i]), int(sp[i]), int(dp[i]), key=key)
            assert qq[i] == O.rss_core(int(sip[i]), int(dip[i]), int(sp[i]), int(dp[i]), 12, 1,
                                       key=key)
    finally:
        ctx.set_rss(None, 1, 0)


def test_rss_arguments_rejected(torch_dev, ctx):
    with pytest.raises(gpucsum.GcsError):
        ctx.set_rss(None, 0, 0)
    with pytest.raises(gpucsum.GcsError):
        ctx.set_rss(b"short", 4, 0)


@pytest.mark.parametrize("frame_len", [100, 576, 1500])
def test_fixed_classify_ip_options_mixed_waves(torch_dev, ctx, O, frame_len):
    """RSS tuple reads: waves whose frames all have ihl = 5 read the tuple at
    fixed lanes; a wave holding one frame with IP options takes the general
    gather.  Options on a whole run of frames (whole waves) and on scattered
    single frames (mixed waves), all against the oracle."""
    t = torch_dev
    n = 8192
    buf, stride = synth.fixed_frames(n, frame_len, seed=frame_len + 5)
    off = np.arange(n, dtype=np.uint64) * stride
    lens = np.full(n, frame_len, dtype=np.uint16)
    rng = np.random.default_rng(frame_len)
    opt = rng.random(n) < 0.02
    opt[1024:1152] = True
    with_opts = 0
    for i in np.nonzero(opt)[0]:
        ihl = int(rng.integers(6, 16))
        if 14 + 4 * ihl + 20 > frame_len:
            continue
        o = int(off[i])
        buf[o + 14] = 0x40 | ihl
        buf[o + 14 + 4 * ihl + 12] = 5 << 4
        with_opts += 1
    O.compute_batch(buf, off, lens)
    ctx.set_rss(None, 16, 0)
    try:
        rvd, rh, rq = O.classify_fixed(buf.copy(), stride, frame_len, n, 16, 0)
        v = zeros(t, n, t.uint8)
        h = zeros(t, n, t.int32)
        q = zeros(t, n, t.int16)
        ctx.classify_fixed(dev(t, buf), stride, frame_len, n, v, h, q)
        ctx.sync()
        np.testing.assert_array_equal(host(v), rvd)
        np.testing.assert_array_equal(host(h).view(np.uint32), rh)
        np.testing.assert_array_equal(host(q).view(np.uint16), rq)
        assert (rvd == 0).all() and with_opts > 100
    finally:
        ctx.set_rss(None, 1, 0)
