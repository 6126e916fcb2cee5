"""Parity of the HIP path (through the C ABI) with the oracle and with the
reference's golden vectors.  Bit-exact: this is integer/byte work.

Runs on a real MI355X (`-m gpu`).  The oracle (oracle/liboracle_csum.so) is
the checker only; every result under test comes from libmtcp_gpucsum.so.
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


# ---------------------------------------------------------------------------
# golden vectors from the reference itself

def test_golden_tcp_fn(torch_dev, ctx):
    t = torch_dev
    d = load("tcp_fn")
    n = len(d["off"])
    out = t.zeros(n, dtype=t.int16, device="cuda")
    ctx.tcp_checksum(dev(t, d["buf"]), dev(t, d["off"].view(np.int64)), dev(t, d["len"].view(np.int16)),
                     dev(t, d["saddr"].view(np.int32)), dev(t, d["daddr"].view(np.int32)), n, out)
    ctx.sync()
    np.testing.assert_array_equal(host(out).view(np.uint16), d["expect"])


def test_golden_ip_fn(torch_dev, ctx):
    t = torch_dev
    d = load("ip_fn")
    n = len(d["off"])
    out = t.zeros(n, dtype=t.int16, device="cuda")
    ctx.ip_checksum(dev(t, d["buf"]), dev(t, d["off"].view(np.int64)), dev(t, d["ihl"]), n, out)
    ctx.sync()
    np.testing.assert_array_equal(host(out).view(np.uint16), d["expect"])


@pytest.mark.parametrize("flags", [0, 1])
def test_golden_frames_rx(torch_dev, ctx, O, flags):
    t = torch_dev
    d = load("frames_rx")
    n = len(d["off"])
    buf = dev(t, d["buf"])
    v = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.verify(buf, dev(t, d["off"].view(np.int64)), dev(t, d["len"].view(np.int16)), n, v,
               flags=flags)
    ctx.sync()
    np.testing.assert_array_equal(host(v), d["expect"])
    # tcp_in.c:1237 side effect, exactly as the oracle applies it
    ref = d["buf"].copy()
    O.verify_batch(ref, d["off"], d["len"], flags=flags)
    np.testing.assert_array_equal(host(buf), ref)


def test_golden_frames_tx(torch_dev, ctx):
    t = torch_dev
    d = load("frames_tx")
    n = len(d["off"])
    buf = dev(t, d["buf"])
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute(buf, dev(t, d["off"].view(np.int64)), dev(t, d["len"].view(np.int16)), n, st, cs)
    ctx.sync()
    np.testing.assert_array_equal(host(st), d["status"])
    np.testing.assert_array_equal(host(cs).view(np.uint32), d["csums"])
    assert hashlib.sha256(host(buf).tobytes()).digest() == d["filled_sha256"].tobytes()


# ---------------------------------------------------------------------------
# fixed-stride kernels: every (G, U) dispatch class vs the oracle

FIXED_LENS = [54, 60, 64, 100, 128, 200, 256, 400, 576, 900, 1024, 1500, 1514, 2000, 4000, 9000]


@pytest.mark.parametrize("frame_len", FIXED_LENS)
def test_fixed_compute_then_verify(torch_dev, ctx, O, frame_len):
    t = torch_dev
    n = 3000 if frame_len < 4000 else 600
    buf, stride = synth.fixed_frames(n, frame_len, seed=frame_len)
    ref = buf.copy()
    rst, rcs = O.compute_fixed(ref, stride, frame_len, n)
    d = dev(t, buf)
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute_fixed(d, stride, frame_len, n, st, cs)
    ctx.sync()
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)
    assert (rst == 0).all()
    # corrupt ~1/8 of the frames, then verify both ways
    bad = synth.corrupt(ref, np.arange(n, dtype=np.uint64) * stride, np.full(n, frame_len),
                        frac_log2=3, seed=frame_len + 1)
    d = dev(t, ref)
    v = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.verify_fixed(d, stride, frame_len, n, v)
    ctx.sync()
    rv = O.verify_fixed(ref, stride, frame_len, n)
    np.testing.assert_array_equal(host(v), rv)
    assert (rv[bad] != 0).all() and (np.delete(rv, bad) == 0).all()


def test_fixed_no_inplace_and_null_outputs(torch_dev, ctx, O):
    t = torch_dev
    n, L = 2048, 1500
    buf, stride = synth.fixed_frames(n, L, seed=5)
    d = dev(t, buf)
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute_fixed(d, stride, L, n, None, cs, flags=K["GCS_CF_NO_INPLACE"])
    ctx.sync()
    np.testing.assert_array_equal(host(d), buf)            # untouched
    ref = buf.copy()
    _, rcs = O.compute_fixed(ref, stride, L, n)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    ctx.compute_fixed(d, stride, L, n)                     # no status, no csums
    ctx.sync()
    np.testing.assert_array_equal(host(d), ref)


# ---------------------------------------------------------------------------
# descriptor kernels: IMIX and fuzzed frames

def test_imix_packed(torch_dev, ctx, O):
    t = torch_dev
    n = 200_000
    lens = synth.imix_lengths(n, seed=3)
    buf, off, lens = synth.packed_frames(lens, seed=4)
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens)
    d = dev(t, buf)
    doff, dlen = dev(t, off.view(np.int64)), dev(t, lens.view(np.int16))
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute(d, doff, dlen, n, st, cs)
    ctx.sync()
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)
    bad = synth.corrupt(ref, off, lens, frac_log2=5, seed=9)
    d = dev(t, ref)
    v = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.verify(d, doff, dlen, n, v)
    ctx.sync()
    rv = O.verify_batch(ref, off, lens)
    np.testing.assert_array_equal(host(v), rv)
    assert (rv[bad] != 0).all()


def fuzz_frames(n, seed):
    """Random headers: every field that steers the verdict is drawn from a
    small set of interesting values, lengths are arbitrary (incl. odd)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 1600, size=n).astype(np.uint16)
    lens[rng.integers(0, n, n // 10)] = rng.integers(0, 80, n // 10)
    off, total = synth.packed_offsets(lens, 16)
    buf = rng.integers(0, 256, size=total + 64, dtype=np.uint8)
    for i in range(n):
        o, L = int(off[i]), int(lens[i])
        f = buf[o:o + max(L, 64)]
        if rng.random() < 0.9:
            f[12], f[13] = 0x08, 0x00
        ihl = int(rng.choice([5, 5, 5, 6, 15, 4, 0, int(rng.integers(0, 16))]))
        ver = 4 if rng.random() < 0.9 else int(rng.integers(0, 16))
        f[14] = (ver << 4) | ihl
        tot = int(rng.choice([L - 14, L - 14, L - 13, L - 15, 19, 20, int(rng.integers(0, 2000))]))
        tot = max(0, min(tot, 65535))
        f[16], f[17] = tot >> 8, tot & 0xFF
        f[23] = 6 if rng.random() < 0.9 else int(rng.integers(0, 256))
        ts = 14 + 4 * ihl
        if ts + 13 < len(f):
            f[ts + 12] = int(rng.choice([5, 8, 15, 0, int(rng.integers(0, 16))])) << 4
    return buf, off, lens


def test_fuzz_desc_vs_oracle(torch_dev, ctx, O):
    t = torch_dev
    n = 20000
    buf, off, lens = fuzz_frames(n, seed=17)
    # make half of them internally consistent so TCP folds are exercised
    tmp = buf.copy()
    O.compute_batch(tmp, off, lens)
    sel = np.random.default_rng(1).random(n) < 0.5
    for i in np.nonzero(sel)[0]:
        o, L = int(off[i]), int(lens[i])
        buf[o:o + L] = tmp[o:o + L]
    d = dev(t, buf)
    doff, dlen = dev(t, off.view(np.int64)), dev(t, lens.view(np.int16))
    v = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.verify(d, doff, dlen, n, v, flags=1)
    ctx.sync()
    ref = buf.copy()
    rv = O.verify_batch(ref, off, lens, flags=1)
    np.testing.assert_array_equal(host(v), rv)
    np.testing.assert_array_equal(host(d), ref)
    assert len(np.unique(rv)) >= 8
    # TX on the same fuzz
    d = dev(t, buf)
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute(d, doff, dlen, n, st, cs)
    ctx.sync()
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens)
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)


def stream_case_frames(n, align, seed, jumbo=0.0, dense_block=None):
    """Packed TCP frames for the prefix-sum stream kernel (k_desc_stream):
    mostly fast frames (ihl 5, te == len, any length incl. odd), plus ihl 6-8
    (fast, general masks), ihl 9-15 (slow list), te < len with padding (slow
    when te > 64), and segments ending inside the first 64 B."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(54, 1515, size=n).astype(np.uint16)
    lens[rng.random(n) < 0.4] = 64
    m = rng.random(n) < 0.1
    lens[m] = rng.integers(54, 80, size=int(m.sum()))
    pj = np.full(n, jumbo)
    if dense_block is not None:
        pj[256 * dense_block:256 * dense_block + 256] = 0.3
    m = rng.random(n) < pj                        # long segments (a block may exceed the region cap)
    lens[m] = rng.integers(1515, 9001, size=int(m.sum()))
    off, total = synth.packed_offsets(lens, align)
    buf = rng.integers(0, 256, size=total + 64, dtype=np.uint8)
    kinds = rng.choice(8, size=n, p=[0.55, 0.08, 0.06, 0.06, 0.07, 0.06, 0.06, 0.06])
    for i in range(n):
        o, L = int(off[i]), int(lens[i])
        f = buf[o:o + L]
        k = int(kinds[i])
        ihl = {1: 6, 2: 7, 3: 8, 4: int(rng.integers(9, 16))}.get(k, 5)
        ts = 14 + 4 * ihl
        if ts + 20 > L:
            ihl, ts = 5, 34
        tot = L - 14
        if k == 5:
            tot = max(4 * ihl + 20, L - 14 - int(rng.integers(1, 40)))     # padded: te < len
        elif k == 6:
            tot = max(4 * ihl + 20, min(L - 14, int(rng.integers(40, 51))))  # te <= 64
        elif k == 7 and L > 64:
            tot = min(L - 14, 64 - 14)                                         # te == 64 < len
        f[12], f[13] = 0x08, 0x00
        f[14] = 0x40 | ihl
        f[16], f[17] = tot >> 8, tot & 0xFF
        f[23] = 6 if rng.random() > 0.03 else 17                            # some IP-only
        f[24] = f[25] = 0
        f[ts + 12] = 5 << 4
        f[ts + 16] = f[ts + 17] = 0
    return buf, off, lens


@pytest.mark.parametrize("align,jumbo", [(16, 0.0), (64, 0.0), (16, 0.015)])
def test_desc_stream_paths_vs_oracle(torch_dev, ctx, O, align, jumbo):
    """Every path of the stream kernel against the oracle, bit-exact: fast
    frames (constant and general masks, Q(te) - Q(64) for te == len), the slow
    list, and whole blocks that fall back to the class passes (a gap > 64 B,
    descriptors out of order, an empty frame)."""
    t = torch_dev
    n = 256 * 24 + 77                                # a partial last block
    buf, off, lens = stream_case_frames(n, align, seed=align + int(jumbo * 1000), jumbo=jumbo,
                                        dense_block=10 if jumbo else None)
    if jumbo:   # block 10 spans more than the stream's region cap (12,288 chunks): class passes
        assert ((lens[2560:2816].astype(int) + 15) // 16).sum() > 12288
    off = off.copy()
    # block 3: one gap > 64 B (frames shifted up by 128 B from frame 3*256+10 on)
    off[3 * 256 + 10:] += 128
    buf = np.concatenate([buf, np.zeros(128, np.uint8)])
    src = buf.copy()
    for i in range(3 * 256 + 10, n):
        o, L = int(off[i]), int(lens[i])
        buf[o:o + L] = src[o - 128:o - 128 + L]
    # block 5: two descriptors swapped (out of offset order)
    a, b = 5 * 256 + 7, 5 * 256 + 8
    off[a], off[b] = off[b], off[a]
    lens[a], lens[b] = lens[b], lens[a]
    # block 7: an empty frame
    lens[7 * 256 + 3] = 0
    doff, dlen = dev(t, off.view(np.int64)), dev(t, lens.view(np.int16))
    # TX
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens)
    d = dev(t, buf)
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute(d, doff, dlen, n, st, cs)
    ctx.sync()
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)
    assert len(np.unique(rst)) >= 3
    # RX, with and without the tcp_in.c:1237 side effect, after corruption
    bad = synth.corrupt(ref, off, np.maximum(lens, 15), frac_log2=3, seed=align + 1)
    for flags in (0, 1):
        d = dev(t, ref)
        v = t.full((n,), 0xEE, dtype=t.uint8, device="cuda")
        ctx.verify(d, doff, dlen, n, v, flags=flags)
        ctx.sync()
        exp = ref.copy()
        rv = O.verify_batch(exp, off, lens, flags=flags)
        np.testing.assert_array_equal(host(v), rv)
        np.testing.assert_array_equal(host(d), exp)
        assert (rv[bad[lens[bad] > 0]] != 0).any()


def test_desc_no_inplace_and_null_outputs(torch_dev, ctx, O):
    """Descriptor batches (the stream kernel and its fallback blocks):
    GCS_CF_NO_INPLACE leaves the frames untouched and still returns the checks;
    a fill with no status / csum outputs still fills in place."""
    t = torch_dev
    n = 256 * 6 + 5
    buf, off, lens = stream_case_frames(n, 64, seed=77)
    off = off.copy()
    a, b = 2 * 256 + 3, 2 * 256 + 4                  # block 2 falls back (descriptors swapped)
    off[a], off[b] = off[b], off[a]
    lens[a], lens[b] = lens[b], lens[a]
    doff, dlen = dev(t, off.view(np.int64)), dev(t, lens.view(np.int16))
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens)
    d = dev(t, buf)
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute(d, doff, dlen, n, st, cs, flags=K["GCS_CF_NO_INPLACE"])
    ctx.sync()
    np.testing.assert_array_equal(host(d), buf)
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    ctx.compute(d, doff, dlen, n)
    ctx.sync()
    np.testing.assert_array_equal(host(d), ref)


def mtu_frames(n, seed, lens=None):
    """Packed (16 B-aligned) TCP frames of 1400-1514 B, all "fast" (ihl 5,
    te == len), checks zeroed."""
    rng = np.random.default_rng(seed)
    if lens is None:
        lens = rng.integers(1400, 1515, size=n).astype(np.uint16)
    off, total = synth.packed_offsets(lens, 16)
    buf = rng.integers(0, 256, size=total + 64, dtype=np.uint8)
    for i in range(n):
        set_tcp_headers(buf, int(off[i]), int(lens[i]), 5, int(lens[i]) - 14)
    return buf, off, lens


def set_tcp_headers(buf, o, L, ihl, tot):
    f = buf[o:o + L]
    ts = 14 + 4 * ihl
    f[12], f[13], f[14] = 0x08, 0x00, 0x40 | ihl
    f[16], f[17] = tot >> 8, tot & 0xFF
    f[23] = 6
    f[24] = f[25] = 0
    f[ts + 12] = 5 << 4
    f[ts + 16] = f[ts + 17] = 0


def test_desc_stream_passes_vs_oracle(torch_dev, ctx, O):
    """Block regions longer than one pass (RMAX chunks): 256 packed MTU frames
    stream in three passes, one workgroup each (blockIdx.y).  A frame that is
    not fast sends its pass and what follows to the per-frame path; frames
    past the last pass go there too.  Bit-exact against the oracle, TX and RX
    (with and without the tcp_in.c:1237 side effect)."""
    t = torch_dev
    n = 256 * 6 + 50
    rng = np.random.default_rng(0x9A55)
    lens = rng.integers(1400, 1515, size=n).astype(np.uint16)
    lens[2 * 256:2 * 256 + 9] = 9000                 # block 2: more than three passes
    buf, off, lens = mtu_frames(n, 0x9A56, lens)
    set_tcp_headers(buf, int(off[256 + 200]), int(lens[256 + 200]), 12,
                    int(lens[256 + 200]) - 14)        # block 1, pass 3: IP options
    i = 3 * 256 + 120                                 # block 3, pass 2: padded (te < len)
    set_tcp_headers(buf, int(off[i]), int(lens[i]), 5, int(lens[i]) - 14 - 30)
    doff, dlen = dev(t, off.view(np.int64)), dev(t, lens.view(np.int16))
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens)
    d = dev(t, buf)
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute(d, doff, dlen, n, st, cs, flags=K["GCS_CF_NO_INPLACE"])
    ctx.sync()
    np.testing.assert_array_equal(host(d), buf)                 # untouched
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    st.zero_()
    cs.zero_()
    ctx.compute(d, doff, dlen, n, st, cs)
    ctx.sync()
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)
    bad = synth.corrupt(ref, off, lens, frac_log2=3, seed=0x9A57)
    for flags in (0, 1):
        d = dev(t, ref)
        v = t.full((n,), 0xEE, dtype=t.uint8, device="cuda")
        ctx.verify(d, doff, dlen, n, v, flags=flags)
        ctx.sync()
        exp = ref.copy()
        rv = O.verify_batch(exp, off, lens, flags=flags)
        np.testing.assert_array_equal(host(v), rv)
        np.testing.assert_array_equal(host(d), exp)
        assert (rv[bad] != 0).all()


def test_desc_mtu_batch_not_serialised(torch_dev, ctx, O):
    """A descriptor batch of 256 x 1500 B frames per block (three passes of
    the stream each, plus a frame per block on the per-frame path): bit-exact
    against the oracle, and not serialised -- the first round-4 form listed
    non-streaming blocks behind one atomic head for a second kernel and took
    22 ms per 1M frames (here: 256K frames in well under 3 ms)."""
    t = torch_dev
    n, L = 1 << 18, 1500
    src, stride = synth.fixed_frames(n, L, seed=0xFB)
    off = np.arange(n, dtype=np.uint64) * stride
    lens = np.full(n, L, dtype=np.uint16)
    doff, dlen = dev(t, off.view(np.int64)), dev(t, lens.view(np.int16))
    ref = src.copy()
    rst, rcs = O.compute_batch(ref, off, lens)
    d = dev(t, src)
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute(d, doff, dlen, n, st, cs)
    ctx.sync()
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)
    bad = synth.corrupt(ref, off, lens, frac_log2=5, seed=0xFC)
    d = dev(t, ref)
    v = t.full((n,), 0xEE, dtype=t.uint8, device="cuda")
    ms = []
    for _ in range(3):
        e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
        e0.record()
        ctx.verify(d, doff, dlen, n, v, stream=t.cuda.current_stream().cuda_stream)
        e1.record()
        t.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    rv = O.verify_batch(ref.copy(), off, lens)
    np.testing.assert_array_equal(host(v), rv)
    assert (rv[bad] != 0).all() and int((rv != 0).sum()) == len(bad)
    assert min(ms) < 3.0, ms


@pytest.mark.parametrize("rooms", [False, True], ids=["stream", "rooms_hint"])
def test_desc_sparse_rooms_vs_oracle(torch_dev, ctx, O, rooms):
    """Frames one per 2 KiB room, as mbufs hand them over (dpdk_module.c's
    rings): no block streams, so every frame takes the stream kernel's
    per-frame path (TX 32 x 2, RX 32 x 3 at 7 waves per SIMD) -- or, with the
    rooms hint (GCS_VF_ROOMS / GCS_CF_ROOMS), the 32-lane group kernel with
    line write-back.  Mixed lengths (empty, runts, odd, MTU, jumbo past one
    batch of 96 chunks), IP options, padded segments and UDP frames, TX and
    RX (with and without the tcp_in.c:1237 side effect) bit-exact against the
    oracle."""
    hint = gpucsum.K["GCS_VF_ROOMS"] if rooms else 0
    t = torch_dev
    n, room = 256 * 5 + 33, 2048
    rng = np.random.default_rng(0x5A2E)
    lens = rng.integers(60, 1515, size=n).astype(np.uint16)
    lens[::97] = 0
    lens[5::89] = rng.integers(1, 54, size=len(lens[5::89]))
    lens[7::211] = rng.integers(1537, 2049, size=len(lens[7::211]))   # > one batch
    off = np.arange(n, dtype=np.uint64) * room
    buf = rng.integers(0, 256, size=n * room, dtype=np.uint8)
    for i in range(n):
        L = int(lens[i])
        if L < 54:
            continue
        ihl = 5 if rng.random() > 0.1 else int(rng.integers(6, 16))
        if 14 + 4 * ihl + 20 > L:
            ihl = 5
        tot = L - 14
        if rng.random() < 0.1:                                   # Ethernet padding
            tot = max(4 * ihl + 20, tot - int(rng.integers(1, 40)))
        set_tcp_headers(buf, int(off[i]), L, ihl, tot)
        if rng.random() < 0.03:
            buf[int(off[i]) + 23] = 17
    doff, dlen = dev(t, off.view(np.int64)), dev(t, lens.view(np.int16))
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens)
    assert len(np.unique(rst)) >= 3
    d = dev(t, buf)
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute(d, doff, dlen, n, st, cs, flags=hint)
    ctx.sync()
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)
    synth.corrupt(ref, off, np.maximum(lens, 15), frac_log2=3, seed=0x5A2F)
    for flags in (0, 1):
        d = dev(t, ref)
        v = t.full((n,), 0xEE, dtype=t.uint8, device="cuda")
        ctx.verify(d, doff, dlen, n, v, flags=flags | hint)
        ctx.sync()
        exp = ref.copy()
        rv = O.verify_batch(exp, off, lens, flags=flags)
        np.testing.assert_array_equal(host(v), rv)
        np.testing.assert_array_equal(host(d), exp)
        assert len(np.unique(rv)) >= 3


@pytest.mark.parametrize("sector_wb", [False, True], ids=["line_wb", "sector_wb"])
def test_rooms_hint_is_only_a_hint(torch_dev, ctx, O, sector_wb):
    """GCS_VF_ROOMS / GCS_CF_ROOMS change the kernel, never the result: packed
    IMIX frames in shuffled descriptor order (neighbouring frames share lines,
    so the line write-back of one frame's group must not clobber another's
    bytes), ragged n, and bad descriptors (misaligned, past the end, length
    over the end) -- TX and RX bit-exact against the oracle, with line and
    with sector write-back (GCS_CF_SECTOR_WB)."""
    t = torch_dev
    n = 3 * 256 + 45
    lens = synth.imix_lengths(n, seed=0x700D)
    buf, off, lens = synth.packed_frames(lens, seed=0x700E)
    perm = np.random.default_rng(0x700F).permutation(n)
    off, lens = off[perm].copy(), lens[perm].copy()
    nb = len(buf)
    off[11], lens[11] = off[11] + 8, 64                 # misaligned
    off[97], lens[97] = (nb + 127) & ~15, 60            # past the end
    off[300], lens[300] = (nb - 48) & ~15, 1500         # length over the end
    hint = gpucsum.K["GCS_CF_ROOMS"] | (gpucsum.K["GCS_CF_SECTOR_WB"] if sector_wb else 0)
    doff, dlen = dev(t, off.view(np.int64)), dev(t, lens.view(np.int16))
    ref = buf.copy()
    rst, rcs = O.compute_batch(ref, off, lens)
    assert (rst == 9).sum() == 3
    d = dev(t, buf)
    st = t.full((n,), 0xEE, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute(d, doff, dlen, n, st, cs, flags=hint)
    ctx.sync()
    np.testing.assert_array_equal(host(st), rst)
    np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
    np.testing.assert_array_equal(host(d), ref)
    good = np.array([i for i in range(n) if i not in (11, 97, 300)])
    synth.corrupt(ref, off[good], np.maximum(lens[good], 15), frac_log2=3, seed=0x7010)
    for flags in (0, 1):
        d = dev(t, ref)
        v = t.full((n,), 0xEE, dtype=t.uint8, device="cuda")
        ctx.verify(d, doff, dlen, n, v, flags=flags | gpucsum.K["GCS_VF_ROOMS"])
        ctx.sync()
        exp = ref.copy()
        rv = O.verify_batch(exp, off, lens, flags=flags)
        np.testing.assert_array_equal(host(v), rv)
        np.testing.assert_array_equal(host(d), exp)
        assert len(np.unique(rv)) >= 3


def test_desc_stream_region_at_buffer_end(torch_dev, ctx, O):
    """A streaming block whose region ends exactly at frames_bytes (16 B-
    aligned: streamed; not aligned: the block falls back to guarded loads)."""
    t = torch_dev
    lens = synth.imix_lengths(300, seed=8)
    lens[-1] = 1504
    buf, off, lens = synth.packed_frames(lens, seed=9)
    for last in (1504, 1497):
        L = lens.copy()
        L[-1] = last
        nb = int(off[-1]) + int(L[-1])
        raw = buf[:nb].copy()
        raw[int(off[-1]) + 16] = (L[-1] - 14) >> 8
        raw[int(off[-1]) + 17] = (L[-1] - 14) & 0xFF
        ref = raw.copy()
        rst, rcs = O.compute_batch(ref, off, L)
        d = dev(t, raw)
        st = t.zeros(len(L), dtype=t.uint8, device="cuda")
        cs = t.zeros(len(L), dtype=t.int32, device="cuda")
        ctx.compute(d, dev(t, off.view(np.int64)), dev(t, L.view(np.int16)), len(L), st, cs,
                    frames_bytes=nb)
        ctx.sync()
        np.testing.assert_array_equal(host(st), rst)
        np.testing.assert_array_equal(host(cs).view(np.uint32), rcs)
        np.testing.assert_array_equal(host(d), ref)
        v = t.full((len(L),), 0xEE, dtype=t.uint8, device="cuda")
        ctx.verify(d, dev(t, off.view(np.int64)), dev(t, L.view(np.int16)), len(L), v,
                   frames_bytes=nb)
        ctx.sync()
        assert (host(v) == 0).all()


def test_bad_descriptors(torch_dev, ctx):
    t = torch_dev
    buf = t.zeros(4096, dtype=t.uint8, device="cuda")
    off = np.array([8, 4096, 4032, 0, 1 << 40], dtype=np.uint64)     # misaligned, at end, past end
    lens = np.array([60, 1, 100, 0, 60], dtype=np.uint16)
    v = t.full((5,), 255, dtype=t.uint8, device="cuda")
    ctx.verify(buf, dev(t, off.view(np.int64)), dev(t, lens.view(np.int16)), 5, v)
    st = t.full((5,), 255, dtype=t.uint8, device="cuda")
    ctx.compute(buf, dev(t, off.view(np.int64)), dev(t, lens.view(np.int16)), 5, st)
    ctx.sync()
    assert host(v).tolist() == [9, 9, 9, 8, 9]
    assert host(st).tolist() == [9, 9, 9, 2, 9]


def test_descriptor_at_buffer_end_is_safe(torch_dev, ctx, O):
    """A frame ending exactly at frames_bytes (not a multiple of 16) must be
    read without touching bytes past the end (guarded partial chunk)."""
    t = torch_dev
    buf, stride = synth.fixed_frames(1, 1500, seed=2)
    O.compute_fixed(buf, stride, 1500, 1)
    raw = buf[:1500].copy()
    d = dev(t, raw)
    v = t.zeros(1, dtype=t.uint8, device="cuda")
    ctx.verify(d, dev(t, np.zeros(1, np.int64)), dev(t, np.array([1500], np.int16)), 1, v,
               frames_bytes=1500)
    ctx.sync()
    assert host(v)[0] == 0


def test_zero_frames_and_invalid_args(torch_dev, ctx):
    t = torch_dev
    buf = t.zeros(64, dtype=t.uint8, device="cuda")
    v = t.zeros(1, dtype=t.uint8, device="cuda")
    ctx.verify_fixed(buf, 64, 64, 0, v)          # n = 0 is a no-op
    with pytest.raises(gpucsum.GcsError):
        ctx.verify_fixed(buf, 48, 64, 1, v)       # stride < frame_len
    with pytest.raises(gpucsum.GcsError):
        ctx.verify_fixed(buf, 72, 64, 1, v)       # stride % 16 != 0
    with pytest.raises(gpucsum.GcsError):
        ctx.verify_fixed(buf, 64, 64, 2, v)       # buffer too small (host check)
    with pytest.raises(gpucsum.GcsError):
        ctx.verify_fixed(np.zeros(64, np.uint8), 64, 64, 1, v)   # host buffer refused


# ---------------------------------------------------------------------------
# host-memory entry points (staged through pinned memory)

def test_host_batches_chunked(torch_dev, O):
    n = 5000
    lens = synth.imix_lengths(n, seed=21)
    buf, off, lens = synth.packed_frames(lens, seed=22)
    with gpucsum.Context(0, max_frames=700, max_bytes=300_000) as c:   # forces many chunks
        b1 = buf.copy()
        st, cs = c.compute_host(b1, off, lens)
        ref = buf.copy()
        rst, rcs = O.compute_batch(ref, off, lens)
        np.testing.assert_array_equal(st, rst)
        np.testing.assert_array_equal(cs, rcs)
        np.testing.assert_array_equal(b1, ref)
        bad = synth.corrupt(ref, off, lens, frac_log2=4, seed=5)
        b2 = ref.copy()
        v = c.verify_host(b2, off, lens, flags=1)
        rv = O.verify_batch(ref, off, lens, flags=1)
        np.testing.assert_array_equal(v, rv)
        np.testing.assert_array_equal(b2, ref)
        assert (rv[bad] != 0).all()


@pytest.mark.parametrize("direct,spread,stage", [(0, 1, "host"), (1 << 30, 0, "host"),
                                                 (1 << 30, 1, "host"), (1 << 30, 1, "device"),
                                                 (1 << 30, 0, "device")])
@pytest.mark.parametrize("n", [1, 64, 700])
def test_host_bursts_direct_and_dma(torch_dev, O, monkeypatch, direct, spread, stage, n):
    """Small host batches (an mTCP burst) through both staging modes: DMA
    copies, and direct mode (the kernel reads the staging in place) on the
    mixed and the spread descriptor kernel, staged in pinned host memory or
    (GCS_DIRECT_STAGE=device) in device memory written over the BAR; jumbo
    frames included."""
    monkeypatch.setenv("GCS_DIRECT_MAX_BYTES", str(direct))
    monkeypatch.setenv("GCS_DIRECT_SPREAD", str(spread))
    monkeypatch.setenv("GCS_DIRECT_STAGE", stage)
    lens = synth.imix_lengths(n, seed=41 + n)
    if n > 1:
        lens[n // 2] = 9000
    buf, off, lens = synth.packed_frames(lens, seed=42 + n)
    with gpucsum.Context(0, max_frames=1024, max_bytes=4 << 20) as c:
        b1 = buf.copy()
        st, cs = c.compute_host(b1, off, lens)
        ref = buf.copy()
        rst, rcs = O.compute_batch(ref, off, lens)
        np.testing.assert_array_equal(st, rst)
        np.testing.assert_array_equal(cs, rcs)
        np.testing.assert_array_equal(b1, ref)
        bad = synth.corrupt(ref, off, lens, frac_log2=2, seed=7)
        for flags in (1, 0):
            b2 = ref.copy()
            v = c.verify_host(b2, off, lens, flags=flags)
            r2 = ref.copy()
            rv = O.verify_batch(r2, off, lens, flags=flags)
            np.testing.assert_array_equal(v, rv)
            np.testing.assert_array_equal(b2, r2)
        assert (rv[bad] != 0).all()


@pytest.mark.parametrize("mode", ["pinned", "registered"])
def test_host_batches_zero_copy(torch_dev, O, mode):
    """Pinned / registered host frames take the span (zero host copy) path."""
    import ctypes as C
    n = 20000
    lens = synth.imix_lengths(n, seed=31)
    buf, off, lens = synth.packed_frames(lens, seed=32)
    if mode == "pinned":
        pb = gpucsum.PinnedBuffer(buf.nbytes)
        host = pb.array
        host[:] = buf
    else:
        host = buf.copy()
        gpucsum.check(gpucsum.lib().gcs_host_register(host.ctypes.data, host.nbytes))
    try:
        with gpucsum.Context(0, max_frames=3000, max_bytes=1 << 20) as c:
            st, cs = c.compute_host(host, off, lens)
            ref = buf.copy()
            rst, rcs = O.compute_batch(ref, off, lens)
            np.testing.assert_array_equal(st, rst)
            np.testing.assert_array_equal(cs, rcs)
            np.testing.assert_array_equal(host, ref)
            bad = synth.corrupt(ref, off, lens, frac_log2=4, seed=6)
            host[:] = ref
            v = c.verify_host(host, off, lens, flags=1)
            rv = O.verify_batch(ref, off, lens, flags=1)
            np.testing.assert_array_equal(v, rv)
            np.testing.assert_array_equal(host, ref)
            assert (rv[bad] != 0).all()
    finally:
        if mode == "pinned":
            pb.free()
        else:
            gpucsum.check(gpucsum.lib().gcs_host_unregister(host.ctypes.data))


# ---------------------------------------------------------------------------
# BASELINE sizes: size-independent properties

@pytest.mark.parametrize("frame_len,n", [(64, 1 << 20), (1500, 1 << 20)])
def test_full_size_properties(torch_dev, ctx, O, frame_len, n):
    """C1/C2 sizes: TX fill then RX verify accepts everything; seeded
    corruptions are exactly the drops; a fill is idempotent; a sample of
    frames matches the oracle bit for bit."""
    t = torch_dev
    buf, stride = synth.fixed_frames(n, frame_len)
    d = dev(t, buf)
    ctx.compute_fixed(d, stride, frame_len, n)
    v = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.verify_fixed(d, stride, frame_len, n, v)
    ctx.sync()
    assert int((v != 0).sum()) == 0
    filled = host(d)
    cs1 = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute_fixed(d, stride, frame_len, n, None, cs1)     # idempotent
    ctx.sync()
    assert t.equal(d.cpu(), t.from_numpy(filled))
    # sample vs oracle
    idx = np.random.default_rng(0).choice(n, 4096, replace=False)
    sample = np.concatenate([buf[i * stride:(i + 1) * stride] for i in idx])
    _, rcs = O.compute_fixed(sample, stride, frame_len, len(idx))
    np.testing.assert_array_equal(host(cs1).view(np.uint32)[idx], rcs)
    # corruptions
    bad = synth.corrupt(filled, np.arange(n, dtype=np.uint64) * stride, np.full(n, frame_len))
    d = dev(t, filled)
    ctx.verify_fixed(d, stride, frame_len, n, v)
    ctx.sync()
    got = np.nonzero(host(v))[0]
    np.testing.assert_array_equal(got, np.sort(bad))


def test_shards_equal_whole(torch_dev, ctx):
    """Per-GPU sharding is exact: verdicts of contiguous frame
    shards equal the verdicts of the whole batch."""
    t = torch_dev
    n, L = 100_003, 1500
    buf, stride = synth.fixed_frames(n, L, seed=99)
    d = dev(t, buf)
    ctx.compute_fixed(d, stride, L, n)
    ctx.sync()
    filled = host(d)
    filled[np.arange(0, n, 37, dtype=np.int64) * stride + 100] ^= 1
    d = dev(t, filled)
    whole = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.verify_fixed(d, stride, L, n, whole)
    parts = t.zeros(n, dtype=t.uint8, device="cuda")
    for k in range(8):
        lo, hi = n * k // 8, n * (k + 1) // 8
        ctx.verify_fixed(d[lo * stride:hi * stride], stride, L, hi - lo, parts[lo:hi])
    ctx.sync()
    assert t.equal(whole, parts)
    assert int((whole != 0).sum()) == len(range(0, n, 37))


def test_c4_shard_properties(torch_dev, ctx, O):
    """C4's per-GPU shard, 4M x 1500 B (6.4 GB at stride 1536, generated in
    HBM as bench.py does): TX fill then RX verify accepts all; a fill is
    idempotent; 4,096 sampled frames match the oracle bit for bit (checks and
    whole filled frames); seeded corruptions are exactly the drops."""
    t = torch_dev
    n, L = 4 << 20, 1500
    d, stride = synth.fixed_frames_device(n, L, seed=0xC4)
    rows = d.view(n, stride)
    idx = np.sort(np.random.default_rng(4).choice(n, 4096, replace=False))
    tidx = t.from_numpy(idx).cuda()
    sample = rows.index_select(0, tidx).cpu().numpy().reshape(-1)      # unfilled originals
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute_fixed(d, stride, L, n, st, cs)
    v = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.verify_fixed(d, stride, L, n, v)
    ctx.sync()
    assert int((st != 0).sum()) == 0 and int((v != 0).sum()) == 0
    rst, rcs = O.compute_fixed(sample, stride, L, len(idx))
    assert (rst == 0).all()
    np.testing.assert_array_equal(host(cs).view(np.uint32)[idx], rcs)
    np.testing.assert_array_equal(rows.index_select(0, tidx).cpu().numpy().reshape(-1), sample)
    before = d.clone()
    ctx.compute_fixed(d, stride, L, n)                                 # idempotent
    ctx.sync()
    assert t.equal(d, before)
    del before
    # corruptions: one byte in [14, 1500) of every 997th frame plus a seeded set
    rng = np.random.default_rng(44)
    bad = np.unique(np.concatenate([np.arange(5, n, 997), rng.choice(n, 3000, replace=False)]))
    pos = rng.integers(14, L, len(bad))
    flip = rng.integers(1, 256, len(bad))
    flat = t.from_numpy(bad.astype(np.int64) * stride + pos).cuda()
    d[flat] ^= t.from_numpy(flip.astype(np.uint8)).cuda()
    ctx.verify_fixed(d, stride, L, n, v)
    ctx.sync()
    got = t.nonzero(v).flatten().cpu().numpy()
    np.testing.assert_array_equal(got, bad)


def test_c3_imix_full_size(torch_dev, ctx, O):
    """C3 at its BASELINE size, 4M IMIX frames packed at 64 B (1.5 GB generated
    in HBM as bench.py does), through the descriptor kernel: the fill's status
    is OK everywhere and verify then accepts all; a fill is idempotent; 4,096
    sampled frames match the oracle bit for bit (checks and whole filled
    frames); seeded corruptions are exactly the drops."""
    t = torch_dev
    n = 4 << 20
    lens = synth.imix_lengths(n, seed=0xC3)
    d, doff, dlen, total = synth.packed_frames_device(lens, seed=0xC3)
    off = doff.cpu().numpy().view(np.uint64)
    idx = np.sort(np.random.default_rng(3).choice(n, 4096, replace=False))
    # the sampled frames, unfilled, repacked for the oracle
    s_len = lens[idx]
    s_off, s_total = synth.packed_offsets(s_len)
    sample = np.zeros(s_total + 64, dtype=np.uint8)
    host_all = d.cpu().numpy()
    for k, i in enumerate(idx):
        sample[int(s_off[k]):int(s_off[k]) + int(s_len[k])] = \
            host_all[int(off[i]):int(off[i]) + int(s_len[k])]
    del host_all
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute(d, doff, dlen, n, st, cs)
    v = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.verify(d, doff, dlen, n, v)
    ctx.sync()
    assert int((st != 0).sum()) == 0 and int((v != 0).sum()) == 0
    ref = sample.copy()
    rst, rcs = O.compute_batch(ref, s_off, s_len)
    assert (rst == 0).all()
    np.testing.assert_array_equal(host(cs).view(np.uint32)[idx], rcs)
    filled = d.cpu().numpy()
    for k, i in enumerate(idx):
        np.testing.assert_array_equal(filled[int(off[i]):int(off[i]) + int(s_len[k])],
                                      ref[int(s_off[k]):int(s_off[k]) + int(s_len[k])])
    before = d.clone()
    ctx.compute(d, doff, dlen, n)                                      # idempotent
    ctx.sync()
    assert t.equal(d, before)
    del before
    # corruptions: one byte in [14, len) of every 997th frame plus a seeded set
    rng = np.random.default_rng(33)
    bad = np.unique(np.concatenate([np.arange(5, n, 997), rng.choice(n, 3000, replace=False)]))
    pos = (rng.random(len(bad)) * (lens[bad].astype(np.int64) - 14)).astype(np.int64) + 14
    flip = rng.integers(1, 256, len(bad))
    flat = t.from_numpy(off[bad].astype(np.int64) + pos).cuda()
    d[flat] ^= t.from_numpy(flip.astype(np.uint8)).cuda()
    ctx.verify(d, doff, dlen, n, v)
    ctx.sync()
    got = t.nonzero(v).flatten().cpu().numpy()
    np.testing.assert_array_equal(got, bad)
