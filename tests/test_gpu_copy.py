"""SURVEY §8f row 4 on the GPU: SendTCPPacket's payload memcpy and both TX
folds fused into one pass (gcs_compute_copy_dev; tcp_out.c:316-333,
ip_out.c:172), bit-exact against the oracle (memcpy + the pinned fill).
Also the write-back at a buffer end that is not 16 B-aligned.
"""
import numpy as np
import pytest

from mtcp_amd import gpucsum, synth
from oracle_lib import Oracle

pytestmark = pytest.mark.gpu
K = gpucsum.K


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


def segments(n, seed, lens=None):
    """TCP frames with headers written and garbage where the payload goes,
    a source buffer and per-frame source offsets of every alignment."""
    rng = np.random.default_rng(seed)
    if lens is None:
        lens = synth.imix_lengths(n, seed=seed)
    buf, off, lens = synth.packed_frames(lens, seed=seed + 1)
    # IP options / TCP options of every size on a quarter of the frames
    for i in np.nonzero(rng.random(n) < 0.25)[0]:
        o, L = int(off[i]), int(lens[i])
        ihl = int(rng.integers(5, 16))
        doff = int(rng.integers(5, 16))
        if 14 + 4 * (ihl + doff) > L:
            continue
        buf[o + 14] = 0x40 | ihl
        buf[o + 14 + 4 * ihl + 12] = doff << 4
    src_bytes = int(lens.astype(np.int64).sum()) + 4096
    src = rng.integers(0, 256, size=src_bytes, dtype=np.uint8)
    src_off = rng.integers(0, src_bytes - 1600, size=n).astype(np.uint64)
    return buf, off, lens, src, src_off


def run_copy(t, ctx, buf, off, lens, src, src_off, frames_bytes=None):
    n = len(off)
    d = dev(t, buf)
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    cs = t.zeros(n, dtype=t.int32, device="cuda")
    ctx.compute_copy(d, dev(t, off.view(np.int64)), dev(t, lens.view(np.int16)), dev(t, src),
                     dev(t, src_off.view(np.int64)), n, st, cs, frames_bytes=frames_bytes)
    ctx.sync()
    return host(d), host(st), host(cs).view(np.uint32)


def test_copy_fill_vs_oracle(torch_dev, ctx, O):
    t = torch_dev
    n = 30000
    buf, off, lens, src, src_off = segments(n, 5)
    # some frames are not complete TCP segments (ICMP, short tot_len): plain fill
    rng = np.random.default_rng(6)
    for i in np.nonzero(rng.random(n) < 0.05)[0]:
        buf[int(off[i]) + 23] = 1
    for i in np.nonzero(rng.random(n) < 0.03)[0]:
        buf[int(off[i]) + 17] ^= 0x40
    got, st, cs = run_copy(t, ctx, buf, off, lens, src, src_off)
    ref = buf.copy()
    rst, rcs = O.compute_copy_batch(ref, off, lens, src, src_off)
    np.testing.assert_array_equal(st, rst)
    np.testing.assert_array_equal(cs, rcs)
    np.testing.assert_array_equal(got, ref)
    assert (rst == 0).mean() > 0.85 and {0, 1, 4} <= set(rst.tolist())
    # copied frames verify clean on the GPU and carry the source bytes
    v = torch_dev.zeros(n, dtype=torch_dev.uint8, device="cuda")
    ctx.verify(dev(t, got), dev(t, off.view(np.int64)), dev(t, lens.view(np.int16)), n, v)
    ctx.sync()
    assert (host(v)[rst == 0] == 0).all()


def test_copy_fill_jumbo_vs_oracle(torch_dev, ctx, O):
    """Frames longer than one batch of the kernel's lanes (> 1536 B, up to
    9014 B jumbo frames): later batches are built before batch 0."""
    t = torch_dev
    n = 3000
    rng = np.random.default_rng(91)
    lens = rng.integers(1400, 9015, size=n).astype(np.uint16)
    lens[::5] = 1536
    lens[1::5] = 1537
    buf, off, lens, src, src_off = segments(n, 91, lens=lens)
    # payloads laid end to end in the source, every alignment
    src_off[:] = np.cumsum(lens.astype(np.uint64)) - lens.astype(np.uint64)
    src_off += rng.integers(0, 16, size=n).astype(np.uint64)
    got, st, cs = run_copy(t, ctx, buf, off, lens, src, src_off)
    ref = buf.copy()
    rst, rcs = O.compute_copy_batch(ref, off, lens, src, src_off)
    np.testing.assert_array_equal(st, rst)
    np.testing.assert_array_equal(cs, rcs)
    np.testing.assert_array_equal(got, ref)
    assert (rst == 0).mean() > 0.95


@pytest.mark.parametrize("payload", [0, 1, 2, 15, 16, 17, 31, 33, 100, 1434, 1448])
@pytest.mark.parametrize("doff", [5, 8, 15])
def test_copy_fill_payload_edges(torch_dev, ctx, O, payload, doff):
    t = torch_dev
    n = 512
    L = 14 + 20 + 4 * doff + payload
    lens = np.full(n, L, dtype=np.uint16)
    buf, off, lens, src, src_off = segments(n, payload * 17 + doff, lens=lens)
    for o in off:
        buf[int(o) + 14] = 0x45
        buf[int(o) + 34 + 12] = doff << 4
    src_off[:16] = np.arange(16)                       # every source alignment
    src_off[16] = len(src) - payload                   # source range ending at the buffer end
    got, st, cs = run_copy(t, ctx, buf, off, lens, src, src_off)
    ref = buf.copy()
    rst, rcs = O.compute_copy_batch(ref, off, lens, src, src_off)
    np.testing.assert_array_equal(st, rst)
    np.testing.assert_array_equal(cs, rcs)
    np.testing.assert_array_equal(got, ref)
    assert (rst == 0).all()
    hl = 34 + 4 * doff
    for k in (0, 7, 16):
        o, so = int(off[k]), int(src_off[k])
        np.testing.assert_array_equal(got[o + hl:o + L], src[so:so + payload])


def test_copy_fill_bad_source_and_buffer_end(torch_dev, ctx, O):
    t = torch_dev
    n = 300
    lens = synth.imix_lengths(n, seed=77)
    lens[-1] = 1501                                    # ends the buffer off a 16 B boundary
    buf, off, lens, src, src_off = segments(n, 77, lens=lens)
    src_off[::7] = len(src) - 3                        # payload would run past the source
    src_off[1::13] = len(src) + 5                      # offset past the source
    # the last frame ends exactly at frames_bytes, which is not 16 B-aligned
    fb = int(off[-1]) + int(lens[-1])
    assert fb % 16
    sentinel = buf.copy()
    sentinel[fb:] = 0xAB
    got, st, cs = run_copy(t, ctx, sentinel, off, lens, src, src_off, frames_bytes=fb)
    ref = sentinel.copy()
    rst, rcs = O.compute_copy_batch(ref[:fb], off, lens, src, src_off)
    np.testing.assert_array_equal(st, rst)
    np.testing.assert_array_equal(cs, rcs)
    np.testing.assert_array_equal(got, ref)
    assert (got[fb:] == 0xAB).all()
    assert K["GCS_TX_BAD_DESC"] in set(rst.tolist())


def test_fill_at_unaligned_buffer_end_writes_nothing_past_it(torch_dev, ctx, O):
    """gcs_compute_dev / gcs_verify_dev on a frame that ends exactly at a
    frames_bytes that is not a multiple of 16: the sector write-back must not
    touch the bytes behind it."""
    t = torch_dev
    for L in (54, 60, 77, 1500, 1501):
        buf, off, lens = synth.packed_frames(np.array([64, L], dtype=np.uint16), seed=L)
        fb = int(off[-1]) + L
        b = buf.copy()
        b[fb:] = 0xAB
        d = dev(t, b)
        st = t.zeros(2, dtype=t.uint8, device="cuda")
        ctx.compute(d, dev(t, off.view(np.int64)), dev(t, lens.view(np.int16)), 2, st,
                    frames_bytes=fb)
        ctx.sync()
        ref = b.copy()
        rst, _ = O.compute_batch(ref[:fb], off, lens)
        got = host(d)
        np.testing.assert_array_equal(host(st), rst)
        np.testing.assert_array_equal(got, ref)
        assert (got[fb:] == 0xAB).all(), L


def test_copy_fill_rejects_flags(torch_dev, ctx):
    t = torch_dev
    z = t.zeros(64, dtype=t.uint8, device="cuda")
    o = t.zeros(1, dtype=t.int64, device="cuda")
    ln = t.full((1,), 64, dtype=t.int16, device="cuda")
    with pytest.raises(gpucsum.GcsError):
        ctx.compute_copy(z, o, ln, z, o, 1, flags=K["GCS_CF_NO_INPLACE"])
