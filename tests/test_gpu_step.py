"""gcs_step_fixed_dev: one launch for the TX fill of one fixed-stride batch and
the RX verify of another (mTCP's loop folds both every iteration,
core.c:761-877).  Results must equal the oracle's -- the TX fill of
ip_out.c:143-173 / tcp_out.c:323-333 and the RX verdicts of ip_in.c:21-59 /
tcp_in.c:1208-1241, with the tcp_in.c:1237 side effect -- for every kernel
shape, the fused launch and its two-launch fallback (different shapes, ICMP
flags, an empty side), and at the C2 size (1M x 1500 B each) the fused
launch must equal the two separate launches byte for byte."""
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


@pytest.mark.parametrize("tx_len,rx_len", [(100, 100), (333, 333), (576, 576), (1024, 1024),
                                           (1500, 1500), (1514, 1500), (2001, 2001),
                                           (9000, 9000), (1500, 333), (64, 1500), (1500, 64)])
@pytest.mark.parametrize("rx_flags", [0, 1])
def test_step_matches_oracle(torch_dev, ctx, tx_len, rx_len, rx_flags):
    t = torch_dev
    O = Oracle()
    n_tx, n_rx = 3001, 2999
    tx, stride_t = synth.fixed_frames(n_tx, tx_len, seed=tx_len)
    rx, stride_r = synth.fixed_frames(n_rx, rx_len, seed=rx_len + 5)
    roff = np.arange(n_rx, dtype=np.uint64) * stride_r
    rlens = np.full(n_rx, rx_len, dtype=np.uint16)
    O.compute_batch(rx, roff, rlens)
    bad = synth.corrupt(rx, roff, rlens, frac_log2=3, seed=rx_len + 6)
    ref_tx, ref_rx = tx.copy(), rx.copy()
    rst, rcs = O.compute_fixed(ref_tx, stride_t, tx_len, n_tx)
    rv = O.verify_batch(ref_rx, roff, rlens, flags=rx_flags)
    dtx = t.from_numpy(tx).cuda()
    drx = t.from_numpy(rx).cuda()
    st = t.zeros(n_tx, dtype=t.uint8, device="cuda")
    cs = t.zeros(n_tx, dtype=t.int32, device="cuda")
    v = t.zeros(n_rx, dtype=t.uint8, device="cuda")
    ctx.step_fixed(dtx, stride_t, tx_len, n_tx, drx, stride_r, rx_len, n_rx, v, st, cs,
                   rx_flags=rx_flags)
    ctx.sync()
    np.testing.assert_array_equal(st.cpu().numpy(), rst)
    np.testing.assert_array_equal(cs.cpu().numpy().view(np.uint32), rcs)
    np.testing.assert_array_equal(dtx.cpu().numpy(), ref_tx)
    np.testing.assert_array_equal(v.cpu().numpy(), rv)
    np.testing.assert_array_equal(drx.cpu().numpy(), ref_rx)    # the side effect, exactly
    assert (rv[bad] != 0).all()


def test_step_icmp_flags_and_empty_sides(torch_dev, ctx):
    """ICMP flags take the two launches; an empty side runs the other alone."""
    t = torch_dev
    O = Oracle()
    n, L = 2000, 576
    tx, stride = synth.fixed_frames(n, L, seed=41)
    off = np.arange(n, dtype=np.uint64) * stride
    lens = np.full(n, L, dtype=np.uint16)
    synth.to_icmp(tx, off, lens, np.arange(0, n, 3))
    rx = tx.copy()
    O.compute_batch(rx, off, lens, flags=2)
    synth.corrupt(rx, off, lens, frac_log2=3, seed=42)
    ref_tx, ref_rx = tx.copy(), rx.copy()
    rst, rcs = O.compute_batch(ref_tx, off, lens, flags=2)
    rv = O.verify_batch(ref_rx, off, lens, flags=K["GCS_VF_ICMP"])
    dtx, drx = t.from_numpy(tx).cuda(), t.from_numpy(rx).cuda()
    st = t.zeros(n, dtype=t.uint8, device="cuda")
    v = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.step_fixed(dtx, stride, L, n, drx, stride, L, n, v, st, tx_flags=K["GCS_CF_ICMP"],
                   rx_flags=K["GCS_VF_ICMP"])
    ctx.sync()
    np.testing.assert_array_equal(st.cpu().numpy(), rst)
    np.testing.assert_array_equal(dtx.cpu().numpy(), ref_tx)
    np.testing.assert_array_equal(v.cpu().numpy(), rv)
    # RX only, then TX only
    v2 = t.zeros(n, dtype=t.uint8, device="cuda")
    ctx.step_fixed(0, stride, L, 0, t.from_numpy(rx).cuda(), stride, L, n, v2,
                   rx_flags=K["GCS_VF_ICMP"])
    d3 = t.from_numpy(tx).cuda()
    ctx.step_fixed(d3, stride, L, n, 0, stride, L, 0, 0, tx_flags=K["GCS_CF_ICMP"])
    ctx.sync()
    np.testing.assert_array_equal(v2.cpu().numpy(), rv)
    np.testing.assert_array_equal(d3.cpu().numpy(), ref_tx)


def test_step_refuses_overlapping_batches(torch_dev, ctx):
    t = torch_dev
    buf = t.zeros(64 * 1536 * 2, dtype=t.uint8, device="cuda")
    v = t.zeros(64, dtype=t.uint8, device="cuda")
    base = buf.data_ptr()
    with pytest.raises(gpucsum.GcsError) as e:
        ctx.step_fixed(base, 1536, 1500, 64, base + 1536 * 63, 1536, 1500, 64, v)
    assert e.value.code == K["GCS_EINVAL"]
    ctx.step_fixed(base, 1536, 1500, 64, base + 1536 * 64, 1536, 1500, 64, v)   # adjacent: fine
    ctx.sync()


def test_step_c2_equals_separate_launches(torch_dev, ctx):
    """C2 (1M x 1500 B TX + 1M x 1500 B RX, BASELINE configs[2]): the fused
    launch's filled TX batch, TX statuses and checks, RX verdicts and RX
    batch equal the two separate launches' byte for byte; every corrupted RX
    frame is dropped and every other accepted."""
    t = torch_dev
    n, L = 1 << 20, 1500
    s = t.cuda.Stream()                 # a real stream: kernels and torch ops in one order
    with t.cuda.stream(s):
        run_c2(t, ctx, n, L, s.cuda_stream)
    s.synchronize()


def run_c2(t, ctx, n, L, stream):
    tx, stride = synth.fixed_frames_device(n, L, seed=0xC2)
    rx = tx.clone()
    ctx.compute_fixed(rx, stride, L, n, stream=stream)
    g = t.Generator(device="cuda")
    g.manual_seed(0xC2B)
    pick = t.nonzero(t.randint(0, 1024, (n,), device="cuda", generator=g) == 0)[:, 0]
    pos = t.randint(14, L, (pick.numel(),), device="cuda", generator=g)
    flip = t.randint(1, 256, (pick.numel(),), device="cuda", generator=g).to(t.uint8)
    idx = pick * stride + pos
    rx[idx] = rx[idx] ^ flip
    tx2, rx2 = tx.clone(), rx.clone()
    st1 = t.zeros(n, dtype=t.uint8, device="cuda")
    cs1 = t.zeros(n, dtype=t.int32, device="cuda")
    v1 = t.zeros(n, dtype=t.uint8, device="cuda")
    st2, cs2, v2 = t.zeros_like(st1), t.zeros_like(cs1), t.zeros_like(v1)
    ctx.step_fixed(tx, stride, L, n, rx, stride, L, n, v1, st1, cs1, rx_flags=1, stream=stream)
    ctx.compute_fixed(tx2, stride, L, n, st2, cs2, stream=stream)
    ctx.verify_fixed(rx2, stride, L, n, v2, flags=1, stream=stream)
    assert t.equal(tx, tx2) and t.equal(rx, rx2)
    assert t.equal(st1, st2) and t.equal(cs1, cs2) and t.equal(v1, v2)
    assert int((st1 != 0).sum()) == 0
    assert int((v1 != 0).sum()) == pick.numel() and int((v1[pick] != 0).sum()) == pick.numel()
