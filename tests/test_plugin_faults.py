"""The decorator's GPU-failure semantics (gpucsum_io_module.h, "GPU failures").

The library's test-only GCS_FAULT_INJECT switch makes one entry point fail
(verify_ptrs, compute_ptrs, compute_async, wait) without touching the GPU; a
context made while the variable is set (to anything) looks its value up per
call.  Each test runs the mTCP-shaped loop (tests/plugin/mini_mtcp.c) through
the decorator over a synthetic NIC and checks the counters, what reaches the
synthetic wire, and what mTCP's RX walk receives:

  RX          every frame of a failed burst comes back NULL from get_rptr
              (rx_errors, rx_unverified), as DPDK surfaces a bad hardware
              checksum (dpdk_module.c:536-542);
  TX in place the inner sends the frames with both check fields as mTCP left
              them, 0 (ip_out.c:153, tcp_out.c:323): tx_unfilled_sent;
  TX_EAGER    (netmap-shaped) nothing of a failed flush reaches the wire:
              tx_unfilled_dropped;
  async post  fill-as-you-go turns off; send_pkts fills synchronously, and
              the wire equals the software path's;
  async wait  the posted fills are cancelled: those frames go out unfilled.
After the fault is lifted the same context works normally again.
"""
import ctypes as C

import numpy as np
import pytest

from test_plugin import (GStats, H, P, MINI_NULL, load, rx_run, tx_frames,  # noqa: F401
                         tx_run, vtab)
from test_plugin_shapes import S, TX_EAGER, mini_tx, wire  # noqa: F401


def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("plugin GPU tests need a GPU (no CPU fallback exists)")


class Ctx:
    """A decorated mTCP thread context over `inner`, made with fault injection
    armed (GCS_FAULT_INJECT=none until a test names an entry point)."""

    def __init__(self, H, P, monkeypatch, inner="synth_module_func", caps=None):  # noqa: F811
        _need_gpu()
        monkeypatch.setenv("GCS_FAULT_INJECT", "none")
        self.H, self.P = H, P
        assert P.gpucsum_set_inner(vtab(H, inner)) == 0
        if caps is not None:
            P.gpucsum_set_inner_caps.argtypes = [C.c_uint32, C.c_uint32]
            assert P.gpucsum_set_inner_caps(caps, 0) == 0
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


def unfilled(buf, off, lens):
    """The frames as mini_mtcp's TX loop leaves them when dev_ioctl says the
    device fills them: iph->check and (TCP) tcph->check 0, nothing else."""
    out = []
    for o, L in zip(off, lens):
        f = buf[int(o):int(o) + int(L)].copy()
        f[24] = f[25] = 0
        if f[23] == 6:
            ts = 14 + 4 * (f[14] & 15)
            f[ts + 16] = f[ts + 17] = 0
        out.append(f)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("group", ["0", "16"])
def test_rx_verify_failure_returns_null(H, P, monkeypatch, group):  # noqa: F811
    """A failing RX verify, one batch per burst (group 0) or posted in groups
    (16: the first post of each burst fails): every frame comes back NULL."""
    monkeypatch.setenv("GPUCSUM_RX_GROUP", group)
    d = load("frames_rx")
    n = len(d["off"])
    c = Ctx(H, P, monkeypatch)
    try:
        monkeypatch.setenv("GCS_FAULT_INJECT", "verify_ptrs")
        disp, st = rx_run(H, c.iom, c.ctx, d["buf"].copy(), d["off"], d["len"], 64)
        g = c.stats()
        assert (disp == MINI_NULL).all()               # nothing reaches ProcessPacket
        assert st.rx_errors == n and st.accepted == 0
        assert g.rx_unverified == n and g.rx_errors == n
        assert g.gpu_failures == (n + 63) // 64         # one failed call per burst
        # lifted: the same context verifies again, as the software path does
        monkeypatch.setenv("GCS_FAULT_INJECT", "none")
        sw_disp, sw = rx_run(H, vtab(H, "synth_module_func"), c.ctx, d["buf"].copy(), d["off"],
                             d["len"], 64)
        disp2, st2 = rx_run(H, c.iom, c.ctx, d["buf"].copy(), d["off"], d["len"], 64)
        assert st2.rx_errors == sw.rx_errors and st2.accepted == sw.accepted
        assert c.stats().gpu_failures == g.gpu_failures
    finally:
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("group", ["0", "8"])
def test_tx_inplace_failure_sends_unfilled(H, P, monkeypatch, group):  # noqa: F811
    """Synchronous fill failing (group 0), or every async wait failing (group 8:
    the posted fills are cancelled): the inner sends the frames with zero
    check fields, each counted in tx_unfilled_sent."""
    monkeypatch.setenv("GPUCSUM_TX_GROUP", group)
    buf, off, lens = tx_frames(1000, 41)
    n = len(off)
    c = Ctx(H, P, monkeypatch)
    try:
        monkeypatch.setenv("GCS_FAULT_INJECT", "compute_ptrs" if group == "0" else "wait")
        hw = tx_run(H, c.iom, c.ctx, buf, off, lens, 64)
        g = c.stats()
        exp = unfilled(buf, off, lens)
        assert len(hw) == n
        for a, b in zip(hw, exp):
            np.testing.assert_array_equal(a, b)
        assert g.tx_unfilled_sent == n and g.tx_frames == 0
        assert g.gpu_failures >= (n + 63) // 64
        if group == "8":
            assert g.tx_posts > 0                      # the posts went out; the waits failed
        monkeypatch.setenv("GCS_FAULT_INJECT", "none")
        sw = tx_run(H, vtab(H, "synth_module_func"), c.ctx, buf, off, lens, 64)
        hw2 = tx_run(H, c.iom, c.ctx, buf, off, lens, 64)
        for a, b in zip(hw2, sw):
            np.testing.assert_array_equal(a, b)
        assert c.stats().tx_unfilled_sent == n
    finally:
        c.close()


@pytest.mark.gpu
def test_tx_async_post_failure_falls_back_to_sync_fill(H, P, monkeypatch):  # noqa: F811
    monkeypatch.setenv("GPUCSUM_TX_GROUP", "8")
    buf, off, lens = tx_frames(1000, 42)
    sw = tx_run(H, vtab(H, "synth_module_func"), C.addressof(C.create_string_buffer(64)),
                buf, off, lens, 64)
    c = Ctx(H, P, monkeypatch)
    try:
        monkeypatch.setenv("GCS_FAULT_INJECT", "compute_async")
        hw = tx_run(H, c.iom, c.ctx, buf, off, lens, 64)
        g = c.stats()
        for a, b in zip(hw, sw):
            np.testing.assert_array_equal(a, b)
        assert g.gpu_failures == 1 and g.tx_posts == 0   # the first post failed: async off
        assert g.tx_unfilled_sent == 0 and g.tx_frames == len(off)
    finally:
        c.close()


@pytest.mark.gpu
def test_tx_shadow_failure_withholds_frames(S, P, monkeypatch):  # noqa: F811
    """netmap-shaped inner (TX_EAGER, shadow slots): a failed fill withholds
    the whole flush from the inner; the next flushes go out filled."""
    monkeypatch.setenv("GPUCSUM_TX_GROUP", "0")       # every fill at the flush
    buf, off, lens = tx_frames(600, 43)
    n = len(off)
    ctx = C.create_string_buffer(64)
    assert S.nmshape_reset(None, None, None, 0, 64) == 0
    mini_tx(S, vtab(S, "nmshape_module_func"), C.addressof(ctx), buf, off, lens, 64)
    sw = wire(S)
    c = Ctx(S, P, monkeypatch, inner="nmshape_module_func", caps=TX_EAGER)
    try:
        assert S.nmshape_reset(None, None, None, 0, 64) == 0
        monkeypatch.setenv("GCS_FAULT_INJECT", "compute_ptrs")
        mini_tx(S, c.iom, c.ctx, buf, off, lens, 64)
        g = c.stats()
        assert S.shape_wire_count() == 0                # nothing unfilled on the wire
        assert g.tx_unfilled_dropped == n and g.tx_unfilled_sent == 0
        assert g.gpu_failures >= (n + 63) // 64
        monkeypatch.setenv("GCS_FAULT_INJECT", "none")
        assert S.nmshape_reset(None, None, None, 0, 64) == 0
        mini_tx(S, c.iom, c.ctx, buf, off, lens, 64)
        hw = wire(S)
        assert len(hw) == len(sw)
        for a, b in zip(hw, sw):
            np.testing.assert_array_equal(a, b)
    finally:
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["tx", "rx"])
def test_lost_requests_reported_once(H, P, monkeypatch, path):  # noqa: F811
    """Every async wait fails for one 64-frame burst (fills in groups of 8,
    verifies in groups of 16: the failed burst leaves cancelled requests in
    up to 8 ring slots), then the fault is lifted and a SHORTER burst follows,
    which reuses fewer slots than were cancelled.  Its waits cover the old
    cancelled requests' numbers; they must not report them: the
    second burst is filled / verified exactly as the software path does."""
    monkeypatch.setenv("GPUCSUM_TX_GROUP", "8")
    monkeypatch.setenv("GPUCSUM_RX_GROUP", "16")
    c = Ctx(H, P, monkeypatch)
    try:
        if path == "tx":
            buf, off, lens = tx_frames(200, 44)
            monkeypatch.setenv("GCS_FAULT_INJECT", "wait")
            tx_run(H, c.iom, c.ctx, buf, off[:64], lens[:64], 64)
            g = c.stats()
            assert g.tx_unfilled_sent == 64
            monkeypatch.setenv("GCS_FAULT_INJECT", "none")
            for k0, k1 in ((64, 84), (84, 200)):
                sw = tx_run(H, vtab(H, "synth_module_func"), c.ctx, buf, off[k0:k1],
                            lens[k0:k1], 64)
                hw = tx_run(H, c.iom, c.ctx, buf, off[k0:k1], lens[k0:k1], 64)
                for a, b in zip(hw, sw):
                    np.testing.assert_array_equal(a, b)
            assert c.stats().tx_unfilled_sent == 64
        else:
            d = load("frames_rx")
            buf, off, lens = d["buf"], d["off"], d["len"]
            monkeypatch.setenv("GCS_FAULT_INJECT", "wait")
            disp, st = rx_run(H, c.iom, c.ctx, buf.copy(), off[:64], lens[:64], 64)
            assert (disp == MINI_NULL).all()
            g = c.stats()
            assert g.rx_unverified == 64
            monkeypatch.setenv("GCS_FAULT_INJECT", "none")
            for k0, k1 in ((64, 84), (84, 300)):
                sw_disp, sw = rx_run(H, vtab(H, "synth_module_func"), c.ctx, buf.copy(),
                                     off[k0:k1], lens[k0:k1], 64)
                hw_disp, hw = rx_run(H, c.iom, c.ctx, buf.copy(), off[k0:k1], lens[k0:k1], 64)
                assert hw.rx_errors == sw.rx_errors and hw.accepted == sw.accepted
            assert c.stats().rx_unverified == 64
    finally:
        c.close()
