"""The decorator driven by mTCP's OWN RX/TX code (oracle/_ref/libref_mtcp_stack.so).

oracle/Makefile compiles the reference's eth_in.c, ip_in.c, tcp_in.c, icmp.c,
ip_out.c, tcp_out.c, eth_out.c, arp.c and tcp_util.c in place, without
-DDISABLE_HWCSUM, so every fold is guarded by the I/O module's dev_ioctl
(ip_in.c:28-37, tcp_in.c:1224-1241, ip_out.c:84-101, tcp_out.c:202-214).
oracle/ref_stack_harness.c runs core.c's RX loop (ProcessPacket per frame)
and SendTCPPacketStandalone per TX segment over any io_module_func.

Reference behaviour: the same code over the synthetic NIC module alone (its
dev_ioctl is NULL, so the reference folds in software).  The decorator over
that module must produce the same dispositions, the same rx_errors and
byte-identical frames on the wire -- TCP segments and the ICMP echo replies
icmp.c builds -- on every frame whose checks the reference can evaluate
inside the frame (frames it would read past are undefined there; the GPU
defines them as DROP_TRUNC).
"""
import ctypes as C
import os

import numpy as np
import pytest

from mtcp_amd import synth
from oracle_lib import ROOT, Oracle
from test_plugin import GStats, load, vtab, H, P  # noqa: F401

STACK_SO = os.path.join(ROOT, "oracle", "_ref", "libref_mtcp_stack.so")
MY_IP = 0x0100000A            # 10.0.0.1 as stored in iph->daddr (network order, LE load)
REFS_ACCEPT, REFS_ERROR, REFS_TRUE, REFS_FALSE, REFS_NULL = 0, 1, 2, 3, 5
vp, u32 = C.c_void_p, C.c_uint32

pytestmark = pytest.mark.skipif(not os.path.exists(STACK_SO),
                                reason="oracle/_ref not built (needs /root/reference at build)")


@pytest.fixture(scope="module")
def R():
    L = C.CDLL(STACK_SO)
    L.refs_config.argtypes = [u32]
    L.refs_rx_loop.argtypes = [vp, vp, C.c_int, vp, u32, C.POINTER(C.c_uint64)]
    L.refs_tx_tcp.argtypes = [vp, vp, u32] + [vp] * 11 + [u32]
    L.refs_tx_stream.argtypes = [vp, vp, u32] + [vp] * 8 + [u32] + [vp] * 5 + [u32]
    L.refs_config(MY_IP)
    return L


def rx_set(seed=3):
    """Golden RX frames + IMIX TCP (some corrupted) + ICMP echo requests to
    MY_IP (some with a bad ICMP checksum), packed at 64 B."""
    g = load("frames_rx")
    n = 3000
    lens = synth.imix_lengths(n, seed=seed)
    buf, off, lens = synth.packed_frames(lens, seed=seed + 1)
    rng = np.random.default_rng(seed)
    icmp = rng.choice(n, n // 8, replace=False)
    synth.to_icmp(buf, off, lens, icmp)
    for i in icmp:
        buf[int(off[i]) + 30:int(off[i]) + 34] = np.frombuffer(np.uint32(MY_IP).tobytes(),
                                                                np.uint8)
    Oracle().compute_batch(buf, off, lens, flags=2)          # GCS_CF_ICMP: IP + ICMP checks
    synth.corrupt(buf, off, lens, frac_log2=4, seed=seed + 2)
    # append the golden frames after the synthetic ones
    base = len(buf)
    gb = g["buf"]
    allbuf = np.concatenate([buf, np.zeros((-base) % 64, np.uint8), gb])
    goff = g["off"].astype(np.uint64) + np.uint64(base + (-base) % 64)
    off = np.concatenate([off, goff])
    lens = np.concatenate([lens, g["len"].astype(np.uint16)])
    return allbuf, off, lens


def run_rx(H, R, iom, ctx, buf, off, lens, burst):
    n = len(off)
    H.synth_reset(burst)
    o = np.ascontiguousarray(off, np.uint64)
    ln = np.ascontiguousarray(lens, np.uint16)
    assert H.synth_set_rx(buf.ctypes.data, o.ctypes.data, ln.ctypes.data, n) == 0
    disp = np.zeros(n, np.uint8)
    errs = C.c_uint64()
    assert R.refs_rx_loop(iom, ctx, 0, disp.ctypes.data, n, C.byref(errs)) == n
    return disp, errs.value, tx_wire(H)


def tx_wire(H):
    tmp = np.zeros(2048, np.uint8)
    out = []
    for k in range(H.synth_tx_sent()):
        L = H.synth_tx_frame(k, tmp.ctypes.data)
        out.append(tmp[:L].copy())
    return out


def tx_args(n, seed):
    rng = np.random.default_rng(seed)
    flags = rng.choice(np.array([0x10, 0x18, 0x11, 0x02, 0x12, 0x04, 0x14], np.uint8), n,
                       p=[0.6, 0.2, 0.05, 0.05, 0.04, 0.03, 0.03])
    syn = (flags & 0x02) != 0
    plen = np.where(syn, 0, rng.integers(0, 1449, n)).astype(np.uint16)
    plen[rng.random(n) < 0.3] = 1448
    plen[syn] = 0
    pay = rng.integers(0, 256, int(plen.sum()) + 16, dtype=np.uint8)
    poff = np.zeros(n, np.uint64)
    np.cumsum(plen[:-1], out=poff[1:])
    a = dict(saddr=rng.integers(0, 2**32, n, dtype=np.uint32),
             sport=rng.integers(1, 65536, n).astype(np.uint16),
             daddr=rng.integers(0, 2**32, n, dtype=np.uint32),
             dport=rng.integers(1, 65536, n).astype(np.uint16),
             seq=rng.integers(0, 2**32, n, dtype=np.uint32),
             ack=rng.integers(0, 2**32, n, dtype=np.uint32),
             window=rng.integers(0, 65536, n).astype(np.uint16), flags=flags,
             payload=pay, pay_off=poff, pay_len=plen)
    return a


def run_tx(H, R, iom, ctx, a, burst):
    H.synth_reset(64)
    n = len(a["flags"])
    keys = ("saddr", "sport", "daddr", "dport", "seq", "ack", "window", "flags", "payload",
            "pay_off", "pay_len")
    assert R.refs_tx_tcp(iom, ctx, n, *[a[k].ctypes.data for k in keys], burst) == n
    return tx_wire(H)


def stream_args(n, seed, ns=8):
    """mTCP's data path: n segments over ns established streams, ACK or
    ACK|PSH with payloads of 0..1448 B (30 % full MSS), as
    FlushTCPSendingBuffer sends them (tcp_out.c:560-600)."""
    rng = np.random.default_rng(seed)
    be16 = lambda x: ((x >> 8) | (x << 8)) & 0xFFFF  # noqa: E731
    st = dict(saddr=rng.integers(0, 2**32, ns, dtype=np.uint32),
              sport=be16(rng.integers(1, 65536, ns)).astype(np.uint16),
              daddr=rng.integers(0, 2**32, ns, dtype=np.uint32),
              dport=be16(rng.integers(1, 65536, ns)).astype(np.uint16),
              snd_nxt=rng.integers(0, 2**32, ns, dtype=np.uint32),
              rcv_nxt=rng.integers(0, 2**32, ns, dtype=np.uint32),
              rcv_wnd=rng.integers(0, 1 << 24, ns, dtype=np.uint32),
              ts_recent=rng.integers(0, 2**32, ns, dtype=np.uint32))
    plen = rng.integers(0, 1449, n).astype(np.uint16)
    plen[rng.random(n) < 0.3] = 1448
    plen[rng.random(n) < 0.1] = 0                                   # pure ACKs
    flags = np.where(rng.random(n) < 0.3, 0x18, 0x10).astype(np.uint8)
    pay = rng.integers(0, 256, int(plen.sum()) + 16, dtype=np.uint8)
    poff = np.zeros(n, np.uint64)
    np.cumsum(plen[:-1], out=poff[1:])
    seg = dict(sidx=rng.integers(0, ns, n).astype(np.uint16), flags=flags, payload=pay,
               pay_off=poff, pay_len=plen)
    return st, seg


def run_tx_stream(H, R, iom, ctx, st, seg, burst):
    H.synth_reset(64)
    n = len(seg["flags"])
    sk = ("saddr", "sport", "daddr", "dport", "snd_nxt", "rcv_nxt", "rcv_wnd", "ts_recent")
    gk = ("sidx", "flags", "payload", "pay_off", "pay_len")
    assert R.refs_tx_stream(iom, ctx, len(st["saddr"]), *[st[k].ctypes.data for k in sk], n,
                            *[seg[k].ctypes.data for k in gk], burst) == n
    return tx_wire(H)


# ---------------------------------------------------------------------------
# CPU: the reference code over the software path agrees with the oracle

def test_ref_stack_software_data_path_tx(H, R):  # noqa: F811
    """SendTCPPacket -> IPOutput over the bare module (software folds): every
    segment verifies, carries its stream's tuple, the NOP NOP TS option with
    the stream's ts_recent, and the stream's sequence numbers in order."""
    st, seg = stream_args(600, 31)
    ctx = C.create_string_buffer(64)
    wire = run_tx_stream(H, R, vtab(H, "synth_module_func"), C.addressof(ctx), st, seg, 64)
    assert len(wire) == 600
    lens = np.array([len(w) for w in wire], np.uint16)
    off, total = synth.packed_offsets(lens)
    buf = np.zeros(total + 64, np.uint8)
    for k, w in enumerate(wire):
        buf[int(off[k]):int(off[k]) + len(w)] = w
    assert (Oracle().verify_batch(buf, off, lens) == 0).all()
    nxt = st["snd_nxt"].astype(np.int64).copy()
    for k, w in enumerate(wire):
        j = int(seg["sidx"][k])
        assert w[14] == 0x45 and w[46] >> 4 == 8                      # ihl 5, doff 8
        assert int.from_bytes(w[26:30].tobytes(), "little") == int(st["saddr"][j])
        assert int.from_bytes(w[38:42].tobytes(), "big") == nxt[j] % 2**32
        assert bytes(w[54:56]) == b"\x01\x01" and w[56] == 8 and w[57] == 10
        assert int.from_bytes(w[62:66].tobytes(), "big") == int(st["ts_recent"][j])
        p0 = int(seg["pay_off"][k])
        np.testing.assert_array_equal(w[66:], seg["payload"][p0:p0 + int(seg["pay_len"][k])])
        nxt[j] += int(seg["pay_len"][k])


def test_ref_stack_software_rx_matches_oracle(H, R):  # noqa: F811
    buf, off, lens = rx_set()
    ctx = C.create_string_buffer(64)
    disp, errs, replies = run_rx(H, R, vtab(H, "synth_module_func"), C.addressof(ctx),
                                 buf.copy(), off, lens, 64)
    v = Oracle().verify_batch(buf.copy(), off, lens)
    inb = ~np.isin(v, [8, 9])
    err = np.isin(v, [2, 3, 6, 7])
    np.testing.assert_array_equal(disp[inb] == REFS_ERROR, err[inb])
    np.testing.assert_array_equal(disp[inb] == REFS_ACCEPT, (v == 0)[inb])
    assert len(replies) > 100      # echo replies to the valid ICMP requests


def test_ref_stack_software_tx_is_valid(H, R):  # noqa: F811
    a = tx_args(400, 9)
    ctx = C.create_string_buffer(64)
    wire = run_tx(H, R, vtab(H, "synth_module_func"), C.addressof(ctx), a, 64)
    assert len(wire) == 400
    lens = np.array([len(w) for w in wire], np.uint16)
    off, total = synth.packed_offsets(lens)
    buf = np.zeros(total + 64, np.uint8)
    for k, w in enumerate(wire):
        buf[int(off[k]):int(off[k]) + len(w)] = w
    assert (Oracle().verify_batch(buf, off, lens) == 0).all()


# ---------------------------------------------------------------------------
# GPU: the decorator under the reference's own callers

@pytest.fixture(scope="module")
def D(H, P):  # noqa: F811
    import torch
    if not torch.cuda.is_available():
        pytest.fail("plugin GPU tests need a GPU (no CPU fallback exists)")
    assert P.gpucsum_set_inner(vtab(H, "synth_module_func")) == 0
    buf = C.create_string_buffer(64)
    ctx = C.addressof(buf)
    iom = vtab(P, "gpucsum_module_func")
    assert H.mini_start(iom, ctx) == 0
    yield iom, ctx, buf
    H.mini_stop(iom, ctx)


@pytest.mark.gpu
@pytest.mark.parametrize("burst", [64, 5, 4000])
def test_decorator_under_reference_rx(H, P, R, D, burst):  # noqa: F811
    iom, ctx, _ = D
    buf, off, lens = rx_set(seed=11 + burst)
    sw_ctx = C.create_string_buffer(64)
    d_sw, e_sw, w_sw = run_rx(H, R, vtab(H, "synth_module_func"), C.addressof(sw_ctx),
                              buf.copy(), off, lens, burst)
    before = GStats()
    P.gpucsum_get_stats(ctx, C.byref(before))
    d_hw, e_hw, w_hw = run_rx(H, R, iom, ctx, buf.copy(), off, lens, burst)
    v = Oracle().verify_batch(buf.copy(), off, lens)
    inb = ~np.isin(v, [8, 9])
    errs = lambda d: np.isin(d, [REFS_ERROR, REFS_NULL])  # noqa: E731
    np.testing.assert_array_equal(errs(d_sw)[inb], errs(d_hw)[inb])
    np.testing.assert_array_equal(d_sw[inb & ~errs(d_sw)], d_hw[inb & ~errs(d_hw)])
    assert (d_hw[errs(d_hw)] == REFS_NULL).all()        # dropped in get_rptr, like DPDK
    assert e_sw - errs(d_sw)[~inb].sum() == e_hw - errs(d_hw)[~inb].sum()
    # ICMP echo replies built by icmp.c: IP check by the GPU vs ip_fast_csum
    assert len(w_sw) == len(w_hw) > 0
    for a, b in zip(w_sw, w_hw):
        np.testing.assert_array_equal(a, b)
    after = GStats()
    P.gpucsum_get_stats(ctx, C.byref(after))
    assert after.gpu_failures == before.gpu_failures


@pytest.mark.gpu
@pytest.mark.parametrize("group", ["0", "1", "8", "64", "100"])
@pytest.mark.parametrize("stage", ["host", "device"])
def test_verify_as_you_go_under_reference_rx(H, P, R, monkeypatch, group, stage):  # noqa: F811
    """Verify as you go (GPUCSUM_RX_GROUP): recv_pkts posts the burst in groups
    and returns; mTCP's get_rptr(i) waits for frame i's group only, while
    ProcessPacket runs on the earlier frames and icmp.c's echo replies are
    filled through the same request ring.  Every group size (0: one
    synchronous batch; 100 > the burst: one group) and staging gives the
    reference's own dispositions, rx_errors and wire frames."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("plugin GPU tests need a GPU (no CPU fallback exists)")
    monkeypatch.setenv("GPUCSUM_RX_GROUP", group)
    monkeypatch.setenv("GCS_ASYNC_STAGE", stage)
    buf, off, lens = rx_set(seed=29)
    sw_ctx = C.create_string_buffer(64)
    d_sw, e_sw, w_sw = run_rx(H, R, vtab(H, "synth_module_func"), C.addressof(sw_ctx),
                              buf.copy(), off, lens, 64)
    assert P.gpucsum_set_inner(vtab(H, "synth_module_func")) == 0
    cbuf = C.create_string_buffer(64)
    ctx = C.addressof(cbuf)
    iom = vtab(P, "gpucsum_module_func")
    assert H.mini_start(iom, ctx) == 0
    try:
        d_hw, e_hw, w_hw = run_rx(H, R, iom, ctx, buf.copy(), off, lens, 64)
        st = GStats()
        P.gpucsum_get_stats(ctx, C.byref(st))
    finally:
        H.mini_stop(iom, ctx)
    v = Oracle().verify_batch(buf.copy(), off, lens)
    inb = ~np.isin(v, [8, 9])
    errs = lambda d: np.isin(d, [REFS_ERROR, REFS_NULL])  # noqa: E731
    np.testing.assert_array_equal(errs(d_sw)[inb], errs(d_hw)[inb])
    np.testing.assert_array_equal(d_sw[inb & ~errs(d_sw)], d_hw[inb & ~errs(d_hw)])
    assert e_sw - errs(d_sw)[~inb].sum() == e_hw - errs(d_hw)[~inb].sum()
    assert len(w_sw) == len(w_hw) > 0
    for a, b in zip(w_sw, w_hw):
        np.testing.assert_array_equal(a, b)
    assert st.gpu_failures == 0
    bursts = (len(off) + 63) // 64
    if group == "0":
        assert st.rx_posts == 0
    else:
        assert st.rx_posts >= bursts


@pytest.mark.gpu
@pytest.mark.parametrize("burst", [64, 1, 1000])
def test_decorator_under_reference_tx(H, P, R, D, burst):  # noqa: F811
    iom, ctx, _ = D
    a = tx_args(2000, 20 + burst)
    sw_ctx = C.create_string_buffer(64)
    sw = run_tx(H, R, vtab(H, "synth_module_func"), C.addressof(sw_ctx), a, burst)
    hw = run_tx(H, R, iom, ctx, a, burst)
    assert len(sw) == len(hw) == 2000
    for x, y in zip(sw, hw):
        np.testing.assert_array_equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("burst", [64, 1, 1000])
def test_decorator_under_reference_data_path(H, P, R, D, burst):  # noqa: F811
    """mTCP's data path (SendTCPPacket -> IPOutput, tcp_out.c:223-357,
    ip_out.c:106-175: stream state, timestamp options, payload memcpy) over
    the decorator: wire-identical to the software folds for 2,000 segments."""
    iom, ctx, _ = D
    st, seg = stream_args(2000, 40 + burst)
    sw_ctx = C.create_string_buffer(64)
    sw = run_tx_stream(H, R, vtab(H, "synth_module_func"), C.addressof(sw_ctx), st, seg, burst)
    hw = run_tx_stream(H, R, iom, ctx, st, seg, burst)
    assert len(sw) == len(hw) == 2000
    for x, y in zip(sw, hw):
        np.testing.assert_array_equal(x, y)
