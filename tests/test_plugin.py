"""The io_module plugin (gpucsum_module_func) as mTCP drives it.

A synthetic NIC module (tests/plugin/synth_module.c) stands in for DPDK, and
tests/plugin/mini_mtcp.c restates mTCP's control flow around the checksum
path (core.c RX loop, eth_in/ip_in/tcp_in verify with dev_ioctl, ip_out/
tcp_out fill with dev_ioctl).  The pure software path (inner module alone,
dev_ioctl NULL) is the reference behaviour; the decorator over the same
module must reproduce it: same per-frame dispositions, same rx_errors, and
byte-identical transmitted frames.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from mtcp_amd import gpucsum, synth
from oracle_lib import Oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLUG = os.path.join(ROOT, "tests", "plugin")
HARNESS = os.path.join(PLUG, "libplugin_harness.so")
GOLD = os.path.join(ROOT, "tests", "golden")

MINI_ACCEPT, MINI_ERROR, MINI_RELEASE, MINI_NOT_TCP, MINI_NON_IP, MINI_NULL = range(6)


class Stats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in
                ("rx_packets", "rx_errors", "accepted", "released", "not_tcp", "non_ip")]


class GStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in
                ("rx_frames", "rx_errors", "rx_batches", "tx_frames", "tx_batches",
                 "gpu_failures", "rx_foreign")] + [("device", C.c_int)] + \
                [(k, C.c_uint64) for k in ("rx_inner", "rx_rptr_changed", "tx_inner_full", "tx_posts",
                                           "tx_unfilled_sent", "tx_unfilled_dropped",
                                           "rx_unverified", "rx_posts")]


@pytest.fixture(scope="module")
def H():
    subprocess.run(["make", "-C", PLUG], check=True, stdout=subprocess.DEVNULL)
    L = C.CDLL(HARNESS)
    vp = C.c_void_p
    L.synth_reset.argtypes = [C.c_uint32]
    L.synth_set_rx.argtypes = [vp, vp, vp, C.c_uint32]
    L.synth_tx_sent.restype = C.c_uint32
    L.synth_tx_frame.argtypes = [C.c_uint32, vp]
    L.mini_start.argtypes = [vp, vp]
    L.mini_stop.argtypes = [vp, vp]
    L.mini_ioctl.argtypes = [vp, vp, C.c_int, C.c_int, vp]
    L.mini_ioctl.restype = C.c_int32
    L.mini_vtable_size.restype = C.c_size_t
    L.mini_rx_loop.argtypes = [vp, vp, C.c_int, C.POINTER(Stats), vp, C.c_uint32]
    L.mini_tx.argtypes = [vp, vp, C.c_int, vp, vp, vp, C.c_uint32, C.c_uint32]
    L.mini_tx_timed.argtypes = [vp, vp, C.c_int, vp, vp, vp, C.c_uint32, C.c_uint32, vp, vp]
    L.synth_tx_base.argtypes = [C.POINTER(C.c_uint64)]
    L.synth_tx_base.restype = vp
    return L


@pytest.fixture(scope="module")
def P():
    L = gpucsum.lib()
    L.gpucsum_set_inner.argtypes = [C.c_void_p]
    L.gpucsum_get_stats.argtypes = [C.c_void_p, C.POINTER(GStats)]
    L.gpucsum_rx_verdict.argtypes = [C.c_void_p, C.c_int, C.c_int]
    L.gpucsum_set_rss.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_int,
                                  C.c_int]
    L.gpucsum_rx_queue.argtypes = [C.c_void_p, C.c_int, C.c_int]
    return L


def vtab(lib, name):
    return C.addressof(C.c_char.in_dll(lib, name))


def load(name):
    with np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


def rx_run(H, iom, ctx, buf, off, lens, burst=64):
    n = len(off)
    H.synth_reset(burst)
    H.synth_set_rx(buf.ctypes.data, np.ascontiguousarray(off, np.uint64).ctypes.data,
                   np.ascontiguousarray(lens, np.uint16).ctypes.data, n)
    st = Stats()
    disp = np.zeros(n, dtype=np.uint8)
    got = H.mini_rx_loop(iom, ctx, 0, C.byref(st), disp.ctypes.data, n)
    assert got == n
    return disp, st


def tx_run(H, iom, ctx, buf, off, lens, burst=64):
    H.synth_reset(burst)
    n = len(off)
    assert H.mini_tx(iom, ctx, 0, buf.ctypes.data,
                     np.ascontiguousarray(off, np.uint64).ctypes.data,
                     np.ascontiguousarray(lens, np.uint16).ctypes.data, n, burst) == n
    assert H.synth_tx_sent() == n
    out = []
    tmp = np.zeros(2048, dtype=np.uint8)
    for k in range(n):
        L = H.synth_tx_frame(k, tmp.ctypes.data)
        out.append(tmp[:L].copy())
    return out


def tx_frames(n, seed):
    """TX-shaped frames (check fields 0, as mTCP leaves them): IMIX TCP plus
    some ICMP (IP check only, ip_out.c:90-92) and IP-option frames."""
    lens = synth.imix_lengths(n, seed=seed)
    buf, off, lens = synth.packed_frames(lens, seed=seed + 1)
    rng = np.random.default_rng(seed)
    for i in rng.choice(n, n // 10, replace=False):
        buf[int(off[i]) + 23] = 1                     # ICMP
    return buf, off, lens


# ---------------------------------------------------------------------------
# no GPU needed

def test_vtable_layout(H):
    """11 function pointers in io_module.h:60-72 order; the typedef's
    aligned(__WORDSIZE) places the object on a 64-byte boundary (GCC keeps
    sizeof at 88 for an aligned typedef, exactly as for the reference)."""
    assert H.mini_vtable_size() == 11 * 8
    out = subprocess.run(["nm", "-S", "-D", gpucsum.LIB_PATH], capture_output=True,
                         text=True).stdout
    line = next(ln for ln in out.splitlines() if ln.endswith(" gpucsum_module_func"))
    addr, size = (int(x, 16) for x in line.split()[:2])
    assert size == 88 and addr % 64 == 0


def test_dev_ioctl_contract(H, P):
    """0 = the device does it; -1 = software (dpdk_module.c:925-927)."""
    assert P.gpucsum_set_inner(None) != 0
    assert P.gpucsum_set_inner(vtab(P, "gpucsum_module_func")) != 0
    assert P.gpucsum_set_inner(vtab(H, "synth_module_func")) == 0
    iom = vtab(P, "gpucsum_module_func")
    want = {0x01: 0, 0x02: -1, 0x03: -1, 0x04: 0, 0x05: 0, 0x06: 0, 0x07: 0, 0x08: -1}
    for cmd, rc in want.items():
        assert H.mini_ioctl(iom, None, 0, cmd, None) == rc, hex(cmd)


def test_software_path_matches_golden(H):
    """The harness itself, over the inner module alone (software folds), drops
    exactly the frames the reference counts as errors."""
    d = load("frames_rx")
    ctx = C.create_string_buffer(64)
    iom = vtab(H, "synth_module_func")
    disp, st = rx_run(H, iom, C.addressof(ctx), d["buf"], d["off"], d["len"])
    is_err = np.isin(d["expect"], [2, 3, 6, 7, 8, 9])
    np.testing.assert_array_equal(disp == MINI_ERROR, is_err)
    assert st.rx_errors == is_err.sum()
    assert st.accepted == (d["expect"] == 0).sum()
    assert st.released == (d["expect"] == 4).sum()


def test_software_tx_matches_oracle(H):
    buf, off, lens = tx_frames(500, 3)
    ctx = C.create_string_buffer(64)
    wire = tx_run(H, vtab(H, "synth_module_func"), C.addressof(ctx), buf, off, lens)
    ref = buf.copy()
    st, _ = Oracle().compute_batch(ref, off, lens)
    assert set(np.unique(st)) <= {0, 1}
    for k, w in enumerate(wire):
        o, L = int(off[k]), int(lens[k])
        np.testing.assert_array_equal(w, ref[o:o + L])


# ---------------------------------------------------------------------------
# the decorator on a GPU

@pytest.fixture(scope="module")
def gpu_plugin(H, P):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("plugin GPU tests need a GPU (no CPU fallback exists)")
    assert P.gpucsum_set_inner(vtab(H, "synth_module_func")) == 0
    ctx = C.create_string_buffer(64)
    iom = vtab(P, "gpucsum_module_func")
    assert H.mini_start(iom, C.addressof(ctx)) == 0
    yield iom, C.addressof(ctx)
    H.mini_stop(iom, C.addressof(ctx))


@pytest.mark.gpu
@pytest.mark.parametrize("burst", [64, 1, 700])
def test_decorator_rx_equals_software_path(H, P, gpu_plugin, burst):
    iom, ctx = gpu_plugin
    d = load("frames_rx")
    sw_disp, sw = rx_run(H, vtab(H, "synth_module_func"), ctx, d["buf"].copy(), d["off"],
                         d["len"], burst)
    before = GStats()
    assert P.gpucsum_get_stats(ctx, C.byref(before)) == 0
    hw_disp, hw = rx_run(H, iom, ctx, d["buf"].copy(), d["off"], d["len"], burst)
    err = lambda x: np.isin(x, [MINI_ERROR, MINI_NULL])  # noqa: E731
    np.testing.assert_array_equal(err(sw_disp), err(hw_disp))
    np.testing.assert_array_equal(sw_disp[~err(sw_disp)], hw_disp[~err(hw_disp)])
    assert (hw_disp[err(hw_disp)] == MINI_NULL).all()   # dropped in get_rptr, like DPDK
    assert (sw.rx_errors, sw.accepted, sw.released, sw.not_tcp, sw.non_ip) == \
           (hw.rx_errors, hw.accepted, hw.released, hw.not_tcp, hw.non_ip)
    after = GStats()
    P.gpucsum_get_stats(ctx, C.byref(after))
    assert after.rx_frames - before.rx_frames == len(d["off"])
    assert after.rx_errors - before.rx_errors == hw.rx_errors
    assert after.gpu_failures == 0


@pytest.mark.gpu
@pytest.mark.parametrize("burst", [64, 3, 5000])
def test_decorator_tx_wire_identical(H, P, gpu_plugin, burst):
    iom, ctx = gpu_plugin
    buf, off, lens = tx_frames(3000, 11)
    sw = tx_run(H, vtab(H, "synth_module_func"), ctx, buf, off, lens, burst)
    before = GStats()
    P.gpucsum_get_stats(ctx, C.byref(before))
    hw = tx_run(H, iom, ctx, buf, off, lens, burst)
    assert len(sw) == len(hw)
    for a, b in zip(sw, hw):
        np.testing.assert_array_equal(a, b)
    after = GStats()
    P.gpucsum_get_stats(ctx, C.byref(after))
    assert after.tx_frames - before.tx_frames == len(off)
    assert after.gpu_failures == 0


@pytest.mark.gpu
@pytest.mark.parametrize("group,registered", [("0", False), ("1", False), ("8", False),
                                              ("64", False), ("8", True), ("1", True)])
def test_async_tx_fill_wire_identical(H, P, monkeypatch, group, registered):
    """Fill as you go (GPUCSUM_TX_GROUP): completed frames go to the burst
    server in groups while the mTCP-shaped loop builds the rest; send_pkts
    posts the tail and waits.  The wire equals the software folds' for every
    group size, with the synthetic NIC's TX rooms pageable or registered
    (both staged into device memory by default since round 4, gcs_api.cpp
    async_reg_stage; GCS_ASYNC_REGISTERED=inplace reads registered rooms in
    place over PCIe)."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("plugin GPU tests need a GPU (no CPU fallback exists)")
    monkeypatch.setenv("GPUCSUM_TX_GROUP", group)
    buf, off, lens = tx_frames(3000, 12)
    ctx = C.create_string_buffer(64)
    sw = tx_run(H, vtab(H, "synth_module_func"), C.addressof(ctx), buf, off, lens, 64)
    assert P.gpucsum_set_inner(vtab(H, "synth_module_func")) == 0
    iom = vtab(P, "gpucsum_module_func")
    dctx = C.create_string_buffer(64)
    assert H.mini_start(iom, C.addressof(dctx)) == 0
    base = None
    try:
        H.synth_reset(64)
        if registered:
            nb = C.c_uint64()
            base = H.synth_tx_base(C.byref(nb))
            gpucsum.check(P.gcs_host_register(C.c_void_p(base), nb.value))
        n = len(off)
        assert H.mini_tx(iom, C.addressof(dctx), 0, buf.ctypes.data,
                         np.ascontiguousarray(off, np.uint64).ctypes.data,
                         np.ascontiguousarray(lens, np.uint16).ctypes.data, n, 64) == n
        hw = []
        tmp = np.zeros(2048, dtype=np.uint8)
        for k in range(n):
            L = H.synth_tx_frame(k, tmp.ctypes.data)
            hw.append(tmp[:L].copy())
        st = GStats()
        assert P.gpucsum_get_stats(C.addressof(dctx), C.byref(st)) == 0
    finally:
        if base:
            gpucsum.check(P.gcs_host_unregister(C.c_void_p(base)))
        H.mini_stop(iom, C.addressof(dctx))
    assert len(sw) == len(hw) == 3000
    for a, b in zip(sw, hw):
        np.testing.assert_array_equal(a, b)
    assert st.tx_frames == 3000 and st.gpu_failures == 0
    if group == "0":
        assert st.tx_posts == 0
    else:
        assert st.tx_posts >= 3000 // max(int(group), 64)


@pytest.mark.gpu
def test_decorator_rx_corrupted_imix(H, P, gpu_plugin):
    iom, ctx = gpu_plugin
    n = 4000
    buf, off, lens = synth.packed_frames(synth.imix_lengths(n, seed=8), seed=9)
    Oracle().compute_batch(buf, off, lens)
    bad = synth.corrupt(buf, off, lens, frac_log2=4, seed=10)
    hw_disp, hw = rx_run(H, iom, ctx, buf.copy(), off, lens)
    assert hw.rx_errors == len(bad)
    assert (hw_disp[bad] == MINI_NULL).all()
    assert (np.delete(hw_disp, bad) == MINI_ACCEPT).all()


@pytest.mark.gpu
@pytest.mark.parametrize("nq,endian,own", [(8, 0, 3), (6, 1, 0)])
def test_decorator_rss_steering_check(H, P, gpu_plugin, nq, endian, own):
    """RSS on: the decorator classifies each burst; dispositions are unchanged
    and rx_foreign counts the ACCEPT frames GetRSSCPUCore (rss.c:97-115)
    assigns to another queue than this thread's."""
    iom, ctx = gpu_plugin
    n = 4000
    buf, off, lens = synth.packed_frames(synth.imix_lengths(n, seed=18), seed=19)
    O = Oracle()
    O.compute_batch(buf, off, lens)
    synth.corrupt(buf, off, lens, frac_log2=4, seed=20)
    vd, _, q = O.classify_batch(buf.copy(), off, lens, nq, endian)
    assert P.gpucsum_set_rss(ctx, None, 0, nq, endian, nq) != 0       # own queue out of range
    assert P.gpucsum_set_rss(ctx, None, 0, nq, endian, own) == 0
    try:
        before = GStats()
        P.gpucsum_get_stats(ctx, C.byref(before))
        disp, st = rx_run(H, iom, ctx, buf.copy(), off, lens)
        after = GStats()
        P.gpucsum_get_stats(ctx, C.byref(after))
        acc = vd == 0
        assert st.accepted == acc.sum()
        assert after.rx_foreign - before.rx_foreign == (acc & (q != own)).sum()
        assert 0 < (acc & (q != own)).sum() < acc.sum()
    finally:
        assert P.gpucsum_set_rss(ctx, None, 0, 0, 0, 0) == 0
