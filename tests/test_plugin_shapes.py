"""The decorator over inner modules with the buffer contracts of mTCP's other
backends (tests/plugin/shapes.c): netmap's eager single-buffer TX, PSIO's
chunk ring with partial sends, and DPDK + ENABLELRO's chained mbufs with the
PKT_RX_TCP_LROSEG gather.  As in test_plugin.py, the inner module alone run
by the mTCP-shaped loop (tests/plugin/mini_mtcp.c) is the reference
behaviour, and the decorator over it must be indistinguishable on the wire
and in what mTCP delivers.
"""
import ctypes as C

import numpy as np
import pytest

from mtcp_amd import gpucsum, synth
from oracle_lib import Oracle
from test_plugin import GStats, Stats, load, tx_frames, vtab, H, P  # noqa: F401

MINI_ACCEPT, MINI_ERROR, MINI_RELEASE, MINI_NOT_TCP, MINI_NON_IP, MINI_NULL = range(6)
TX_EAGER, RX_CHAINED, RX_ONCE = 0x1, 0x2, 0x4
vp = C.c_void_p


@pytest.fixture(scope="module")
def S(H, P):  # noqa: F811
    H.nmshape_reset.argtypes = [vp, vp, vp, C.c_uint32, C.c_uint32]
    H.psshape_reset.argtypes = [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32]
    H.psshape_pending.restype = C.c_uint32
    H.psshape_partial_sends.restype = C.c_uint32
    H.lroshape_reset.argtypes = [vp, vp, vp, vp, vp, vp, C.c_uint32, C.c_uint32]
    H.lroshape_gathers.restype = C.c_uint32
    H.dfshape_reset.argtypes = [vp, vp, vp, C.c_uint32, C.c_uint32, vp, vp, vp, vp]
    H.dfshape_refeeds.restype = C.c_uint32
    H.shape_wire_count.restype = C.c_uint32
    H.shape_wire_frame.argtypes = [C.c_uint32, vp]
    H.mini_send.argtypes = [vp, vp, C.c_int]
    H.mini_rx_deliver.argtypes = [vp, vp, C.c_int, C.POINTER(Stats), vp, C.c_uint32, C.c_int,
                                  vp, C.c_uint64, vp, vp]
    P.gpucsum_set_inner_caps.argtypes = [C.c_uint32, C.c_uint32]
    P.gpucsum_get_inner.restype = vp
    return H


def wire(H):
    tmp = np.zeros(2048, dtype=np.uint8)
    out = []
    for k in range(H.shape_wire_count()):
        L = H.shape_wire_frame(k, tmp.ctypes.data)
        out.append(tmp[:L].copy())
    return out


def mini_tx(H, iom, ctx, buf, off, lens, burst):
    assert H.mini_tx(iom, ctx, 0, buf.ctypes.data,
                     np.ascontiguousarray(off, np.uint64).ctypes.data,
                     np.ascontiguousarray(lens, np.uint16).ctypes.data, len(off), burst) == len(off)


class Decorated:
    """gpucsum_module_func over `inner` with `caps`, started like mTCP starts
    a thread's module (core.c:1639, :1190)."""

    def __init__(self, H, P, inner, caps=0, seg_max=0):
        import torch
        if not torch.cuda.is_available():
            pytest.fail("plugin GPU tests need a GPU (no CPU fallback exists)")
        self.H, self.P = H, P
        assert P.gpucsum_set_inner(vtab(H, inner)) == 0
        assert P.gpucsum_get_inner() == vtab(H, inner)
        assert P.gpucsum_set_inner_caps(caps, seg_max) == 0
        self.buf = C.create_string_buffer(64)
        self.ctx = C.addressof(self.buf)
        self.iom = vtab(P, "gpucsum_module_func")
        assert H.mini_start(self.iom, self.ctx) == 0

    def stats(self):
        st = GStats()
        assert self.P.gpucsum_get_stats(self.ctx, C.byref(st)) == 0
        return st

    def close(self):
        self.H.mini_stop(self.iom, self.ctx)


# ---------------------------------------------------------------------------
# CPU: the shapes themselves behave like the backends they stand for

def test_caps_api(S, P):  # noqa: F811
    assert P.gpucsum_set_inner(vtab(S, "nmshape_module_func")) == 0
    assert P.gpucsum_set_inner_caps(0x8, 0) != 0            # unknown cap
    assert P.gpucsum_set_inner_caps(RX_ONCE | RX_CHAINED, 0) != 0   # cur_rx_m (LRO gather)
    assert P.gpucsum_set_inner_caps(RX_ONCE, 0) == 0
    assert P.gpucsum_set_inner_caps(TX_EAGER, 70000) != 0   # seg_max > 65535
    assert P.gpucsum_set_inner_caps(TX_EAGER | RX_CHAINED, 0) == 0
    assert P.gpucsum_get_inner() == vtab(S, "nmshape_module_func")


def test_netmap_shape_sends_on_get_wptr(S):
    """netmap_get_wptr transmits the previous frame (netmap_module.c:155-156):
    with the software path, every frame reaches the wire filled."""
    buf, off, lens = tx_frames(200, 5)
    ctx = C.create_string_buffer(64)
    assert S.nmshape_reset(None, None, None, 0, 64) == 0
    mini_tx(S, vtab(S, "nmshape_module_func"), C.addressof(ctx), buf, off, lens, 64)
    got = wire(S)
    ref = buf.copy()
    Oracle().compute_batch(ref, off, lens)
    assert len(got) == 200
    for k, w in enumerate(got):
        np.testing.assert_array_equal(w, ref[int(off[k]):int(off[k]) + int(lens[k])])


def test_psio_shape_partial_sends(S):
    """ps_send_chunk_buf may move part of the chunk; the rest stays queued for
    the next send_pkts (psio_module.c:213-229)."""
    buf, off, lens = tx_frames(700, 6)
    ctx = C.create_string_buffer(64)
    assert S.psshape_reset(None, None, None, 0, 64, 5) == 0
    mini_tx(S, vtab(S, "psshape_module_func"), C.addressof(ctx), buf, off, lens, 64)
    while S.psshape_pending():
        S.mini_send(vtab(S, "psshape_module_func"), C.addressof(ctx), 0)
    assert S.psshape_partial_sends() > 0
    assert S.shape_wire_count() == 700


# ---------------------------------------------------------------------------
# GPU: the decorator over each shape

@pytest.mark.gpu
@pytest.mark.parametrize("burst", [64, 1, 300])
def test_netmap_tx_wire_identical(S, P, burst):  # noqa: F811
    buf, off, lens = tx_frames(2500, 31)
    ctx = C.create_string_buffer(64)
    assert S.nmshape_reset(None, None, None, 0, 64) == 0
    mini_tx(S, vtab(S, "nmshape_module_func"), C.addressof(ctx), buf, off, lens, burst)
    sw = wire(S)
    d = Decorated(S, P, "nmshape_module_func", TX_EAGER)
    try:
        assert S.nmshape_reset(None, None, None, 0, 64) == 0
        mini_tx(S, d.iom, d.ctx, buf, off, lens, burst)
        hw = wire(S)
        st = d.stats()
    finally:
        d.close()
    assert len(hw) == len(sw) == 2500
    for a, b in zip(sw, hw):
        np.testing.assert_array_equal(a, b)
    assert st.tx_frames == 2500 and st.gpu_failures == 0 and st.tx_inner_full == 0


@pytest.mark.gpu
def test_netmap_in_place_mode_is_detectably_wrong(S, P):  # noqa: F811
    """Control: treating netmap as an in-place module (the round-1 decorator)
    lets frames leave before their fill, so the wire differs."""
    buf, off, lens = tx_frames(300, 32)
    ctx = C.create_string_buffer(64)
    assert S.nmshape_reset(None, None, None, 0, 64) == 0
    mini_tx(S, vtab(S, "nmshape_module_func"), C.addressof(ctx), buf, off, lens, 64)
    sw = wire(S)
    d = Decorated(S, P, "nmshape_module_func", 0)
    try:
        assert S.nmshape_reset(None, None, None, 0, 64) == 0
        mini_tx(S, d.iom, d.ctx, buf, off, lens, 64)
        hw = wire(S)
    finally:
        d.close()
    assert sum(not np.array_equal(a, b) for a, b in zip(sw, hw)) > 250


@pytest.mark.gpu
def test_netmap_rx_equals_software_path(S, P):  # noqa: F811
    g = load("frames_rx")
    ctx = C.create_string_buffer(64)
    disp_sw = np.zeros(len(g["off"]), np.uint8)
    disp_hw = np.zeros_like(disp_sw)
    st_sw, st_hw = Stats(), Stats()
    n = len(g["off"])
    goff = np.ascontiguousarray(g["off"], np.uint64)
    glen = np.ascontiguousarray(g["len"], np.uint16)
    args = (g["buf"].ctypes.data, goff.ctypes.data, glen.ctypes.data, n, 64)
    assert S.nmshape_reset(*args) == 0
    assert S.mini_rx_loop(vtab(S, "nmshape_module_func"), C.addressof(ctx), 0,
                          C.byref(st_sw), disp_sw.ctypes.data, n) == n
    d = Decorated(S, P, "nmshape_module_func", TX_EAGER)
    try:
        assert S.nmshape_reset(*args) == 0
        assert S.mini_rx_loop(d.iom, d.ctx, 0, C.byref(st_hw), disp_hw.ctypes.data, n) == n
    finally:
        d.close()
    err = lambda x: np.isin(x, [MINI_ERROR, MINI_NULL])  # noqa: E731
    np.testing.assert_array_equal(err(disp_sw), err(disp_hw))
    assert (st_sw.rx_errors, st_sw.accepted, st_sw.released) == \
           (st_hw.rx_errors, st_hw.accepted, st_hw.released)


@pytest.mark.gpu
@pytest.mark.parametrize("send_limit", [5, 256])
def test_psio_tx_wire_identical(S, P, send_limit):  # noqa: F811
    buf, off, lens = tx_frames(1500, 41)

    def run(iom, ctx):
        assert S.psshape_reset(None, None, None, 0, 64, send_limit) == 0
        mini_tx(S, iom, ctx, buf, off, lens, 64)
        while S.psshape_pending():
            S.mini_send(iom, ctx, 0)
        return wire(S)

    ctx = C.create_string_buffer(64)
    sw = run(vtab(S, "psshape_module_func"), C.addressof(ctx))
    d = Decorated(S, P, "psshape_module_func", 0)
    try:
        hw = run(d.iom, d.ctx)
        st = d.stats()
    finally:
        d.close()
    assert len(sw) == len(hw) == 1500
    for a, b in zip(sw, hw):
        np.testing.assert_array_equal(a, b)
    assert st.tx_frames == 1500 and st.gpu_failures == 0


@pytest.mark.gpu
def test_psio_rx_chunk_equals_software_path(S, P):  # noqa: F811
    n = 3000
    buf, off, lens = synth.packed_frames(synth.imix_lengths(n, seed=44), seed=45)
    Oracle().compute_batch(buf, off, lens)
    bad = synth.corrupt(buf, off, lens, frac_log2=4, seed=46)
    args = (buf.ctypes.data, off.ctypes.data, lens.ctypes.data, n, 64)
    ctx = C.create_string_buffer(64)
    disp_sw = np.zeros(n, np.uint8)
    disp_hw = np.zeros(n, np.uint8)
    st_sw, st_hw = Stats(), Stats()
    assert S.psshape_reset(*args, 0) == 0
    S.mini_rx_loop(vtab(S, "psshape_module_func"), C.addressof(ctx), 0, C.byref(st_sw),
                   disp_sw.ctypes.data, n)
    d = Decorated(S, P, "psshape_module_func", 0)
    try:
        assert S.psshape_reset(*args, 0) == 0
        S.mini_rx_loop(d.iom, d.ctx, 0, C.byref(st_hw), disp_hw.ctypes.data, n)
    finally:
        d.close()
    assert st_sw.rx_errors == st_hw.rx_errors == len(bad)
    assert st_sw.accepted == st_hw.accepted == n - len(bad)
    assert (disp_hw[bad] == MINI_NULL).all()


def lro_burst(n, seed):
    """A received stream for an ENABLELRO port: single-segment frames (<= 1514
    B, some corrupted so the NIC flags them) and LRO chains of 2..7 segments
    with payloads above TCP_DEFAULT_MSS (some flagged bad by the NIC)."""
    rng = np.random.default_rng(seed)
    chain = rng.random(n) < 0.3
    lens = np.where(chain, rng.integers(3000, 12000, n), synth.imix_lengths(n, seed=seed))
    buf, off, lens = synth.packed_frames(lens.astype(np.uint16), seed=seed + 1)
    single = ~chain
    Oracle().compute_batch(buf, off, lens)          # valid checks on every frame
    orig = buf.copy()
    corrupted = synth.corrupt(buf, off, lens, frac_log2=3, seed=seed + 2)
    for k in np.nonzero(chain)[0]:                  # chains: NIC-merged, intact headers
        o = int(off[k])
        buf[o:o + int(lens[k])] = orig[o:o + int(lens[k])]
    vd = Oracle().verify_batch(buf.copy(), off, lens)
    bad = np.zeros(n, np.uint8)
    err = np.isin(vd, [2, 3, 6, 7, 8, 9])
    bad[single & err] = 1                           # NIC rejects what the reference would
    bad[chain & (rng.random(n) < 0.1)] = 1
    first = rng.integers(200, 1500, n).astype(np.uint16)
    rest = lens.astype(np.int64) - first
    nseg = np.where(chain, 1 + -(-rest // 1900), 1).astype(np.uint8)
    return buf, off, lens.astype(np.uint32), nseg, first, bad, chain, corrupted


@pytest.mark.gpu
@pytest.mark.parametrize("burst", [64, 17])
def test_lro_gathers_the_right_frame(S, P, burst):  # noqa: F811
    """mTCP's ENABLELRO receive path (tcp_ring_buffer.c:15-21 + dpdk_module.c:
    855-881) delivers the same payload bytes through the decorator as through
    the inner module alone: every PKT_RX_TCP_LROSEG gathers the mbuf mTCP is
    processing, because the decorator re-calls the inner get_rptr per index."""
    n = 1200
    buf, off, lens, nseg, first, bad, chain, _ = lro_burst(n, 70)
    args = (buf.ctypes.data, off.ctypes.data, lens.ctypes.data, nseg.ctypes.data,
            first.ctypes.data, bad.ctypes.data, n, burst)
    cap = int(lens.astype(np.int64).sum())

    def run(iom, ctx):
        assert S.lroshape_reset(*args) == 0
        st = Stats()
        disp = np.zeros(n, np.uint8)
        out = np.zeros(cap, np.uint8)
        o = np.zeros(n, np.uint64)
        ln = np.zeros(n, np.uint32)
        assert S.mini_rx_deliver(iom, ctx, 0, C.byref(st), disp.ctypes.data, n, 1,
                                 out.ctypes.data, cap, o.ctypes.data, ln.ctypes.data) == n
        pay = [out[int(o[k]):int(o[k]) + int(ln[k])].copy() if ln[k] else None
               for k in range(n)]
        return st, disp, pay, S.lroshape_gathers()

    ctx = C.create_string_buffer(64)
    st_sw, disp_sw, pay_sw, g_sw = run(vtab(S, "lroshape_module_func"), C.addressof(ctx))
    d = Decorated(S, P, "lroshape_module_func", RX_CHAINED)
    try:
        st_hw, disp_hw, pay_hw, g_hw = run(d.iom, d.ctx)
        gst = d.stats()
    finally:
        d.close()
    np.testing.assert_array_equal(disp_sw, disp_hw)
    assert (st_sw.rx_errors, st_sw.accepted) == (st_hw.rx_errors, st_hw.accepted)
    assert g_sw == g_hw > 0
    # chains the NIC flagged bad were NULL already in the burst pass
    assert gst.rx_inner == (chain & (bad == 0)).sum() and gst.rx_rptr_changed == 0
    for k in range(n):
        if pay_sw[k] is None:
            assert pay_hw[k] is None
            continue
        np.testing.assert_array_equal(pay_sw[k], pay_hw[k])
        # and the gathered bytes are this frame's own payload
        o, L = int(off[k]), int(lens[k])
        ihl = int(buf[o + 14]) & 15
        hl = 14 + 4 * ihl + 4 * (int(buf[o + 14 + 4 * ihl + 12]) >> 4)
        np.testing.assert_array_equal(pay_hw[k], buf[o + hl:o + L])


def defrag_wire(n, seed):
    """An RX wire for an IP_DEFRAG port: plain frames (some corrupted), absorbed
    fragments and completing fragments, each of the latter with the datagram
    the reassembly table hands back (some of those corrupted too)."""
    rng = np.random.default_rng(seed)
    buf, off, lens = synth.packed_frames(synth.imix_lengths(n, seed=seed), seed=seed + 1)
    Oracle().compute_batch(buf, off, lens)
    synth.corrupt(buf, off, lens, frac_log2=3, seed=seed + 2)
    u = rng.random(n)
    frag = np.where(u < 0.15, 1, np.where(u < 0.25, 2, 0)).astype(np.uint8)
    wb, wo, wl = synth.packed_frames(synth.imix_lengths(n, seed=seed + 3), seed=seed + 4)
    Oracle().compute_batch(wb, wo, wl)
    synth.corrupt(wb, wo, wl, frac_log2=2, seed=seed + 5)
    return buf, off, lens, frag, wb, wo, wl


@pytest.mark.gpu
@pytest.mark.parametrize("burst", [64, 9])
def test_defrag_inner_called_once(S, P, burst):  # noqa: F811
    """DPDK with IP_DEFRAG (dpdk_module.c:474-513, 527-529): get_rptr feeds a
    fragment to the reassembly table on every call.  With RX_ONCE the
    decorator calls it once per index and mTCP sees exactly what the inner
    module alone gives it: the same dispositions, rx_errors and reassembled
    datagrams verified on the GPU.  Without it the burst pass's call consumes
    each completing fragment and mTCP's own call re-feeds it (a NULL)."""
    n = 900
    buf, off, lens, frag, wb, wo, wl = defrag_wire(n, 90)
    args = (buf.ctypes.data, off.ctypes.data, lens.ctypes.data, n, burst, frag.ctypes.data,
            wb.ctypes.data, wo.ctypes.data, wl.ctypes.data)

    def run(iom, ctx):
        assert S.dfshape_reset(*args) == 0
        st = Stats()
        disp = np.zeros(n, np.uint8)
        assert S.mini_rx_loop(iom, ctx, 0, C.byref(st), disp.ctypes.data, n) == n
        return st, disp, S.dfshape_refeeds()

    ctx = C.create_string_buffer(64)
    st_sw, disp_sw, rf_sw = run(vtab(S, "dfshape_module_func"), C.addressof(ctx))
    assert rf_sw == 0
    d = Decorated(S, P, "dfshape_module_func", RX_ONCE)
    try:
        st_hw, disp_hw, rf_hw = run(d.iom, d.ctx)
        gst = d.stats()
    finally:
        d.close()
    # a frame the GPU rejects is a NULL from get_rptr, as DPDK's hardware check
    # gives it (dpdk_module.c:536-542): both count as rx_errors (core.c:794-799)
    err = lambda x: np.isin(x, [MINI_ERROR, MINI_NULL])  # noqa: E731
    np.testing.assert_array_equal(err(disp_sw), err(disp_hw))
    np.testing.assert_array_equal(disp_sw == MINI_ACCEPT, disp_hw == MINI_ACCEPT)
    assert (st_sw.rx_errors, st_sw.accepted, st_sw.released) == \
           (st_hw.rx_errors, st_hw.accepted, st_hw.released)
    assert rf_hw == 0 and gst.rx_rptr_changed == 0
    done = frag == 2
    assert (disp_hw[done] == MINI_ACCEPT).sum() > 0 and err(disp_hw[done]).sum() > 0
    # the default (idempotent inner) mode: completing fragments are lost
    d = Decorated(S, P, "dfshape_module_func", 0)
    try:
        st_x, disp_x, rf_x = run(d.iom, d.ctx)
        gx = d.stats()
    finally:
        d.close()
    # every completing fragment the GPU accepted was fed again by mTCP's call
    assert rf_x == gx.rx_rptr_changed > 0
    assert (disp_x[done] == MINI_NULL).all() and st_x.accepted < st_sw.accepted


@pytest.mark.gpu
def test_rx_burst_larger_than_gpu_batch(H, P):  # noqa: F811
    """A recv_pkts burst above GPUCSUM_MAX_BURST (8192) is verified whole."""
    from test_plugin import rx_run
    n = 12000
    buf, off, lens = synth.packed_frames(synth.imix_lengths(n, seed=50), seed=51)
    Oracle().compute_batch(buf, off, lens)
    bad = synth.corrupt(buf, off, lens, frac_log2=5, seed=52)
    d = Decorated(H, P, "synth_module_func", 0)
    try:
        disp, st = rx_run(H, d.iom, d.ctx, buf.copy(), off, lens, burst=n)
        gst = d.stats()
    finally:
        d.close()
    assert st.rx_errors == len(bad) and st.accepted == n - len(bad)
    assert (disp[bad] == MINI_NULL).all()
    assert gst.rx_frames == n and gst.gpu_failures == 0


@pytest.mark.gpu
@pytest.mark.parametrize("burst", [64, 7])
def test_decorator_without_burst_server(H, P, monkeypatch, burst):  # noqa: F811
    """The plugin serves bursts through the resident grid by default (every
    other plugin test runs that way); with GPUCSUM_BURST_SERVER=0 each burst
    is one kernel launch.  Dispositions and wire bytes are the same."""
    from test_plugin import rx_run, tx_run
    monkeypatch.setenv("GPUCSUM_BURST_SERVER", "0")
    g = load("frames_rx")
    buf, off, lens = tx_frames(1500, 77)
    sw_ctx = C.create_string_buffer(64)
    sw_disp, sw = rx_run(H, vtab(H, "synth_module_func"), C.addressof(sw_ctx), g["buf"].copy(),
                         g["off"], g["len"], burst)
    sw_wire = tx_run(H, vtab(H, "synth_module_func"), C.addressof(sw_ctx), buf, off, lens, burst)
    d = Decorated(H, P, "synth_module_func", 0)
    try:
        hw_disp, hw = rx_run(H, d.iom, d.ctx, g["buf"].copy(), g["off"], g["len"], burst)
        hw_wire = tx_run(H, d.iom, d.ctx, buf, off, lens, burst)
        st = d.stats()
    finally:
        d.close()
    err = lambda x: np.isin(x, [MINI_ERROR, MINI_NULL])  # noqa: E731
    np.testing.assert_array_equal(err(sw_disp), err(hw_disp))
    assert (sw.rx_errors, sw.accepted, sw.released) == (hw.rx_errors, hw.accepted, hw.released)
    for a, b in zip(sw_wire, hw_wire):
        np.testing.assert_array_equal(a, b)
    assert st.gpu_failures == 0 and st.tx_frames == 1500
