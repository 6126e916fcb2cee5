"""Failure behaviour of the host-memory entry points (gcs_api.cpp).

The C ABI promises status codes, never C++ exceptions (mtcp_gpucsum.h), and a
failed call must not leave state that corrupts the next one.  Failures are
simulated with the library's test-only GCS_FAULT_INJECT switch:

  gather_thread  the gather pool cannot start its helper threads
                 (std::system_error): the calling thread copies alone;
  gather_alloc   the pool allocation throws std::bad_alloc: GCS_ENOMEM;
  second_chunk   a HIP failure after chunk 1 of a batch was launched: the
                 call fails, and the next call on the same context is exact.
"""
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


def batch(n, seed):
    buf, off, lens = synth.packed_frames(synth.imix_lengths(n, seed=seed), seed=seed + 1)
    Oracle().compute_batch(buf, off, lens)
    bad = synth.corrupt(buf, off, lens, frac_log2=4, seed=seed + 2)
    return buf, off, lens, bad


def test_gather_threads_unavailable(torch_dev, monkeypatch):
    monkeypatch.setenv("GCS_FAULT_INJECT", "gather_thread")
    monkeypatch.setenv("GCS_GATHER_THREADS", "64")
    buf, off, lens, bad = batch(20000, 10)
    # chunks of ~2 MiB (byte-limited): above the 1 MiB inline-gather threshold
    with gpucsum.Context(0, max_frames=1 << 16, max_bytes=4 << 20) as c:
        v = c.verify_host(buf.copy(), off, lens)
    np.testing.assert_array_equal(v, Oracle().verify_batch(buf.copy(), off, lens))
    assert (v[bad] != 0).all()


def test_bad_alloc_is_a_status_code(torch_dev, monkeypatch):
    buf, off, lens, bad = batch(20000, 20)
    with gpucsum.Context(0, max_frames=1 << 16, max_bytes=4 << 20) as c:
        monkeypatch.setenv("GCS_FAULT_INJECT", "gather_alloc")
        with pytest.raises(gpucsum.GcsError) as e:
            c.verify_host(buf.copy(), off, lens)
        assert e.value.code == gpucsum.K["GCS_ENOMEM"]
        assert "bad_alloc" in gpucsum.lib().gcs_last_hip_error().decode()
        monkeypatch.delenv("GCS_FAULT_INJECT")
        v = c.verify_host(buf.copy(), off, lens)
    np.testing.assert_array_equal(v, Oracle().verify_batch(buf.copy(), off, lens))


@pytest.mark.parametrize("compute", [False, True])
def test_failed_batch_leaves_no_busy_slot(torch_dev, monkeypatch, compute):
    """Chunk 1 (513 frames) is in flight when the call fails.  The next call on
    the same context (100 frames) must see none of it: before the fix its first
    drain copied the stale chunk's 513 results into the new call's 100-entry
    arrays, past their end.  The output arrays carry guard bytes here."""
    import ctypes as C
    L = gpucsum.lib()
    b1, off1, len1, _ = batch(6000, 30)
    b2, off2, len2, bad2 = batch(100, 40)
    guard = 4096
    with gpucsum.Context(0, max_frames=1024, max_bytes=1 << 20) as c:
        monkeypatch.setenv("GCS_FAULT_INJECT", "second_chunk")
        with pytest.raises(gpucsum.GcsError):
            if compute:
                c.compute_host(b1.copy(), off1, len1)
            else:
                c.verify_host(b1.copy(), off1, len1)
        monkeypatch.delenv("GCS_FAULT_INJECT")
        out = np.full(100 + guard, 0xAA, np.uint8)
        got = b2.copy()
        if compute:
            got[off2.astype(np.int64)[:, None] + np.array([24, 25, 50, 51])] = 0
            ref = got.copy()
            cs = np.full(100 + guard, 0xAAAAAAAA, np.uint32)
            gpucsum.check(L.gcs_compute(c.h, got.ctypes.data, off2.ctypes.data, len2.ctypes.data,
                                        100, out.ctypes.data, cs.ctypes.data))
            rst, rcs = Oracle().compute_batch(ref, off2, len2)
            np.testing.assert_array_equal(out[:100], rst)
            np.testing.assert_array_equal(cs[:100], rcs)
            np.testing.assert_array_equal(got, ref)
            assert (cs[100:] == 0xAAAAAAAA).all()
        else:
            gpucsum.check(L.gcs_verify(c.h, got.ctypes.data, off2.ctypes.data, len2.ctypes.data,
                                       100, out.ctypes.data, 0))
            np.testing.assert_array_equal(out[:100], Oracle().verify_batch(b2.copy(), off2, len2))
            assert (out[bad2] != 0).all()
        assert (out[100:] == 0xAA).all()


def test_frame_larger_than_staging_is_refused_whole(torch_dev):
    """ERANGE before anything runs: no frame of the batch is touched."""
    lens = synth.imix_lengths(300, seed=5)
    lens[200] = 9000
    buf, off, lens = synth.packed_frames(lens, seed=6)
    orig = buf.copy()
    with gpucsum.Context(0, max_frames=64, max_bytes=8192) as c:   # 4 KiB per slot
        with pytest.raises(gpucsum.GcsError) as e:
            c.compute_host(buf, off, lens)
        assert e.value.code == gpucsum.K["GCS_ERANGE"]
        np.testing.assert_array_equal(buf, orig)
        ok = np.arange(200)
        st, _ = c.compute_host(buf, off[ok], lens[ok])
        assert set(np.unique(st)) <= {0}


# ---------------------------------------------------------------------------
# burst server (gcs_ctx_set_burst_server): resident grid for direct-mode batches

def bursts(n_bursts, n, seed, jumbo=False):
    out = []
    for k in range(n_bursts):
        lens = synth.imix_lengths(n, seed=seed + k)
        if jumbo and n > 2:
            lens[n // 2] = 9000
        buf, off, lens = synth.packed_frames(lens, seed=seed + 100 + k)
        out.append((buf, off, lens))
    return out


@pytest.mark.parametrize("idle_us,life_us,gap_s,stage", [(200, 2000, 0.0, "host"),
                                                         (30, 2000, 0.002, "host"),
                                                         (200, 150, 0.0, "host"),
                                                         (200, 2000, 0.0, "device")])
def test_burst_server_matches_oracle(torch_dev, monkeypatch, idle_us, life_us, gap_s, stage):
    """Bursts through the resident grid, including grids that leave between
    bursts (idle exit: gaps longer than GCS_SERVER_IDLE_US) and in the middle
    of a run (lifetime exit), staged in pinned host or (GCS_DIRECT_STAGE)
    device memory: every burst is exact."""
    import time
    monkeypatch.setenv("GCS_SERVER_IDLE_US", str(idle_us))
    monkeypatch.setenv("GCS_SERVER_LIFE_US", str(life_us))
    monkeypatch.setenv("GCS_DIRECT_STAGE", stage)
    O = Oracle()
    with gpucsum.Context(0, max_frames=1024, max_bytes=4 << 20) as c:
        c.set_burst_server(True)
        for k, (buf, off, lens) in enumerate(bursts(60, 64, 300, jumbo=True)):
            b1 = buf.copy()
            st, cs = c.compute_host(b1, off, lens)
            ref = buf.copy()
            rst, rcs = O.compute_batch(ref, off, lens)
            np.testing.assert_array_equal(st, rst)
            np.testing.assert_array_equal(cs, rcs)
            np.testing.assert_array_equal(b1, ref)
            bad = synth.corrupt(ref, off, lens, frac_log2=2, seed=k)
            v = c.verify_host(ref.copy(), off, lens, flags=1)
            np.testing.assert_array_equal(v, O.verify_batch(ref.copy(), off, lens, flags=1))
            assert (v[bad] != 0).all()
            if gap_s:
                time.sleep(gap_s)


@pytest.mark.parametrize("wait,spin_us,presleep_ns", [("yield", "0", "0"), ("sleep", "0", "0"),
                                                      ("spin", "4", "2000")])
def test_burst_server_wait_policies(torch_dev, monkeypatch, wait, spin_us, presleep_ns):
    """The host's wait policies (GCS_SERVER_WAIT / _SPIN_US / _PRESLEEP_NS,
    read when the context joins the grid) change how a thread waits, never
    what it gets: every burst is exact."""
    monkeypatch.setenv("GCS_SERVER_WAIT", wait)
    monkeypatch.setenv("GCS_SERVER_SPIN_US", spin_us)
    monkeypatch.setenv("GCS_SERVER_PRESLEEP_NS", presleep_ns)
    O = Oracle()
    with gpucsum.Context(0, max_frames=1024, max_bytes=4 << 20) as c:
        c.set_burst_server(True)
        for k, (buf, off, lens) in enumerate(bursts(20, 64, 700)):
            b1 = buf.copy()
            st, cs = c.compute_host(b1, off, lens)
            ref = buf.copy()
            rst, rcs = O.compute_batch(ref, off, lens)
            np.testing.assert_array_equal(st, rst)
            np.testing.assert_array_equal(cs, rcs)
            np.testing.assert_array_equal(b1, ref)
            bad = synth.corrupt(ref, off, lens, frac_log2=2, seed=k)
            v = c.verify_host(ref.copy(), off, lens, flags=1)
            np.testing.assert_array_equal(v, O.verify_batch(ref.copy(), off, lens, flags=1))
            assert (v[bad] != 0).all()


def test_burst_server_yields_to_large_batches(torch_dev):
    """With the server on, a batch too large for direct mode takes the DMA
    path (the grid leaves first), and bursts after it are served again."""
    O = Oracle()
    big = bursts(1, 60000, 900)[0]
    with gpucsum.Context(0, max_frames=1 << 16, max_bytes=8 << 20) as c:
        c.set_burst_server(True)
        for buf, off, lens in bursts(3, 64, 910) + [big] + bursts(3, 64, 920):
            v = c.verify_host(buf.copy(), off, lens)
            np.testing.assert_array_equal(v, O.verify_batch(buf.copy(), off, lens))
        c.set_burst_server(False)
        buf, off, lens = bursts(1, 64, 930)[0]
        v = c.verify_host(buf.copy(), off, lens)
        np.testing.assert_array_equal(v, O.verify_batch(buf.copy(), off, lens))


@pytest.mark.parametrize("server,start,skew,cached", [(False, None, None, False),
                                                      (True, None, None, False),
                                                      (True, None, None, True),
                                                      (False, None, None, True),
                                                      (True, 0x80000002, None, False),
                                                      (True, 0xFFFFFFFF - 4, None, False),
                                                      (True, 0xFFFF0, 0x7FFFFFF0, False)],
                         ids=["direct", "server", "server_cached", "direct_cached",
                              "server_seq_2^31", "server_seq_wrap", "server_stale_ack"])
def test_registered_rooms_in_place(torch_dev, monkeypatch, server, start, skew, cached):
    """Frames in one registered region (an mbuf pool) are verified and filled
    in place over PCIe -- no gather, no scatter -- with the same results; a
    frame outside the region, or misaligned, sends the batch down the staged
    path, also exact.  The server's in-place requests complete on the serving
    blocks' acks; with the request numbers starting >= 2^31 past 0 or at the
    32-bit wrap, an ack the ring joined with at 0 would read as newer than the
    request and complete it before its release: every result must
    still equal the oracle.  server_stale_ack joins the ring with acks 2^31 + 16
    requests behind it (GCS_SERVER_ACK_SKEW), as after 2^31 requests that
    wrote no frame: the grid refreshes them before it serves.
    The region is registered uncached by default (the grid then skips the L2
    invalidate before reading its frames); *_cached registers it cached.
    Every burst rewrites the rooms with new frames, as a NIC reuses mbufs: a
    stale cached line would show as a wrong verdict or check."""
    import ctypes as C
    if cached:
        monkeypatch.setenv("GCS_REGISTER_UNCACHED", "0")
    if start is not None:
        monkeypatch.setenv("GCS_SERVER_SEQ_START", str(start))
    if skew is not None:
        monkeypatch.setenv("GCS_FAULT_INJECT", "ack_skew")      # test-only knob, gated
        monkeypatch.setenv("GCS_SERVER_ACK_SKEW", str(skew))
    L = gpucsum.lib()
    O = Oracle()
    n = 64
    rooms = np.zeros(n * 2048 + 8192, dtype=np.uint8)
    base = (-rooms.ctypes.data) % 4096
    mb = rooms[base:base + n * 2048]
    other = np.zeros(4096, dtype=np.uint8)
    gpucsum.check(L.gcs_host_register(mb.ctypes.data, mb.nbytes))
    try:
        with gpucsum.Context(0, max_frames=1024, max_bytes=4 << 20) as c:
            if server:
                c.set_burst_server(True)
            for k in range(6):
                buf, off, lens = bursts(1, n, 500 + k, jumbo=False)[0]
                lens = lens.copy()
                for i in range(n):
                    mb[i * 2048:i * 2048 + int(lens[i])] = buf[int(off[i]):int(off[i]) + int(lens[i])]
                addrs = [mb.ctypes.data + i * 2048 for i in range(n)]
                if k == 4:                      # one frame outside the region
                    other[:int(lens[3])] = mb[3 * 2048:3 * 2048 + int(lens[3])]
                    addrs[3] = other.ctypes.data
                if k == 5:                      # one misaligned frame
                    mb[9 * 2048 + 2:9 * 2048 + 2 + int(lens[9])] = mb[9 * 2048:9 * 2048 + int(lens[9])].copy()
                    addrs[9] += 2
                ptrs = (C.c_void_p * n)(*addrs)
                frames = [np.ctypeslib.as_array((C.c_uint8 * int(lens[i])).from_address(addrs[i]))
                          for i in range(n)]
                ref_frames = [f.copy() for f in frames]
                st = np.zeros(n, np.uint8)
                cs = np.zeros(n, np.uint32)
                gpucsum.check(L.gcs_compute_ptrs(c.h, ptrs, lens.ctypes.data, n, st.ctypes.data,
                                                 cs.ctypes.data))
                o64, total = synth.packed_offsets(lens)
                pk = np.zeros(total + 64, np.uint8)
                for i in range(n):
                    pk[int(o64[i]):int(o64[i]) + int(lens[i])] = ref_frames[i]
                rst, rcs = O.compute_batch(pk, o64, lens)
                np.testing.assert_array_equal(st, rst)
                np.testing.assert_array_equal(cs, rcs)
                for i in range(n):
                    np.testing.assert_array_equal(frames[i], pk[int(o64[i]):int(o64[i]) + int(lens[i])])
                # corrupt a few and verify in place (tcp_in.c:1237 side effect on)
                for i in (1, 17, 40):
                    frames[i][30] ^= 0x5A
                    pk[int(o64[i]) + 30] ^= 0x5A
                v = np.zeros(n, np.uint8)
                gpucsum.check(L.gcs_verify_ptrs(c.h, ptrs, lens.ctypes.data, n, v.ctypes.data, 1))
                rv = O.verify_batch(pk, o64, lens, flags=1)
                np.testing.assert_array_equal(v, rv)
                for i in range(n):
                    np.testing.assert_array_equal(frames[i], pk[int(o64[i]):int(o64[i]) + int(lens[i])])
                assert (v[[1, 17, 40]] != 0).all()
    finally:
        gpucsum.check(L.gcs_host_unregister(mb.ctypes.data))


@pytest.mark.parametrize("start", [0xFFFF - 3, 0x2FFFF - 2, 0xFFFFFFFF - 4])
def test_burst_server_request_tags_wrap(torch_dev, monkeypatch, start):
    """The per-frame records carry the request number's low 16 bits, and a
    cleared record reads as tag 0: a request tagged 0 would complete at once,
    before the grid read it (every 65536th burst).  Requests are
    numbered across the 16-bit tag boundary and the 32-bit wrap here, on the
    staged paths that complete on the records alone (RX verify, TX fill into
    staging); every burst must equal the oracle."""
    monkeypatch.setenv("GCS_SERVER_SEQ_START", str(start))
    O = Oracle()
    with gpucsum.Context(0, max_frames=1024, max_bytes=4 << 20) as c:
        c.set_burst_server(True)
        for k, (buf, off, lens) in enumerate(bursts(5, 64, 700)):
            b1 = buf.copy()
            st, cs = c.compute_host(b1, off, lens)
            ref = buf.copy()
            rst, rcs = O.compute_batch(ref, off, lens)
            np.testing.assert_array_equal(st, rst)
            np.testing.assert_array_equal(cs, rcs)
            np.testing.assert_array_equal(b1, ref)
            bad = synth.corrupt(ref, off, lens, frac_log2=2, seed=k)
            v = c.verify_host(ref.copy(), off, lens)
            np.testing.assert_array_equal(v, O.verify_batch(ref.copy(), off, lens))
            assert (v[bad] != 0).all()


def test_host_register_refuses_overlap(torch_dev):
    L = gpucsum.lib()
    rooms = np.zeros(3 * 4096, dtype=np.uint8)
    base = (-rooms.ctypes.data) % 4096
    a = rooms.ctypes.data + base
    gpucsum.check(L.gcs_host_register(a, 4096))
    try:
        assert L.gcs_host_register(a, 4096) == gpucsum.K["GCS_EINVAL"]
        assert L.gcs_host_register(a + 2048, 4096) == gpucsum.K["GCS_EINVAL"]
    finally:
        gpucsum.check(L.gcs_host_unregister(a))


@pytest.mark.parametrize("stage", ["host", "device"])
def test_async_fill_many_outstanding(torch_dev, monkeypatch, stage):
    """gcs_compute_ptrs_async: 40 posts of 1..120 frames without waiting (past
    the 8 request slots, so posts finish older fills to reuse a slot), one
    wait on an older ticket, then the last: every status, check and filled
    frame equals the oracle.  GCS_ASYNC_STAGE=device stages in device memory."""
    import ctypes as C
    monkeypatch.setenv("GCS_ASYNC_STAGE", stage)
    L = gpucsum.lib()
    L.gcs_compute_ptrs_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
    L.gcs_wait.argtypes = [C.c_void_p, C.c_uint64]
    buf, off, lens = synth.packed_frames(synth.imix_lengths(2400, seed=61), seed=62)
    ref = buf.copy()
    rst, rcs = Oracle().compute_batch(ref, off, lens)
    ptrs = (C.c_void_p * len(off))(*[buf.ctypes.data + int(o) for o in off])
    st = np.full(len(off), 0xEE, np.uint8)
    cs = np.zeros(len(off), np.uint32)
    rng = np.random.default_rng(63)
    tickets = []
    with gpucsum.Context(0, max_frames=4096, max_bytes=8 << 20) as c:
        c.set_burst_server(True)
        i = 0
        while i < len(off):
            m = min(int(rng.integers(1, 121)), len(off) - i)
            t = C.c_uint64()
            gpucsum.check(L.gcs_compute_ptrs_async(
                c.h, C.cast(C.byref(ptrs, 8 * i), C.c_void_p), lens.ctypes.data + 2 * i, m,
                st.ctypes.data + i, cs.ctypes.data + 4 * i, C.byref(t)))
            assert t.value != 0
            tickets.append(t.value)
            i += m
            if len(tickets) == 20:
                gpucsum.check(L.gcs_wait(c.h, tickets[5]))
        assert len(tickets) >= 25
        gpucsum.check(L.gcs_wait(c.h, tickets[-1]))
    np.testing.assert_array_equal(st, rst)
    np.testing.assert_array_equal(cs, rcs)
    np.testing.assert_array_equal(buf, ref)


@pytest.mark.parametrize("stage,registered", [("host", False), ("device", False),
                                               ("host", True)])
def test_async_verify_interleaved_with_fills(torch_dev, monkeypatch, stage, registered):
    """gcs_verify_ptrs_async (the plugin's RX verify as you go) interleaved
    with gcs_compute_ptrs_async on one context's request ring: 60 posts of
    1..64 frames, alternating at random between verifies of corrupted frames
    and fills of TX frames, past the 8 request slots, waits on older tickets
    in between.  Every verdict -- and the tcp_in.c:1237 side effect on bad TCP
    frames, written by the host at completion -- every status and every filled
    frame equals the oracle.  Frames staged in pinned or device memory, or
    read in place from a registered region."""
    import ctypes as C
    monkeypatch.setenv("GCS_ASYNC_STAGE", stage)
    L = gpucsum.lib()
    L.gcs_verify_ptrs_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                        C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
    L.gcs_compute_ptrs_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
    L.gcs_wait.argtypes = [C.c_void_p, C.c_uint64]
    O = Oracle()
    n = 1800
    rx, roff, rlens = synth.packed_frames(synth.imix_lengths(n, seed=81), seed=82)
    O.compute_batch(rx, roff, rlens)
    bad = synth.corrupt(rx, roff, rlens, frac_log2=3, seed=83)
    tx, toff, tlens = synth.packed_frames(synth.imix_lengths(n, seed=84), seed=85)
    mem = np.zeros(rx.nbytes + tx.nbytes + 16384, np.uint8)
    base = (-mem.ctypes.data) % 4096
    rxm = mem[base:base + rx.nbytes]
    txo = base + rx.nbytes + ((-(base + rx.nbytes)) % 64)
    txm = mem[txo:txo + tx.nbytes]
    rxm[:] = rx
    txm[:] = tx
    rref, tref = rx.copy(), tx.copy()
    rv = O.verify_batch(rref, roff, rlens, flags=1)      # GCS_VF_ZERO_BAD_TCP_CHECK
    rst, rcs = O.compute_batch(tref, toff, tlens)
    rp = (C.c_void_p * n)(*[rxm.ctypes.data + int(o) for o in roff])
    tp = (C.c_void_p * n)(*[txm.ctypes.data + int(o) for o in toff])
    vd = np.full(n, 0xEE, np.uint8)
    st = np.full(n, 0xEE, np.uint8)
    cs = np.zeros(n, np.uint32)
    rng = np.random.default_rng(86)
    if registered:
        gpucsum.check(L.gcs_host_register(mem.ctypes.data + base, (mem.nbytes - base) & ~4095))
    try:
        with gpucsum.Context(0, max_frames=4096, max_bytes=8 << 20) as c:
            c.set_burst_server(True)
            i = j = 0
            tickets = []
            while i < n or j < n:
                t = C.c_uint64()
                if j >= n or (i < n and rng.random() < 0.5):
                    m = min(int(rng.integers(1, 65)), n - i)
                    gpucsum.check(L.gcs_verify_ptrs_async(
                        c.h, C.cast(C.byref(rp, 8 * i), C.c_void_p), rlens.ctypes.data + 2 * i, m,
                        vd.ctypes.data + i, 1, C.byref(t)))
                    i += m
                else:
                    m = min(int(rng.integers(1, 65)), n - j)
                    gpucsum.check(L.gcs_compute_ptrs_async(
                        c.h, C.cast(C.byref(tp, 8 * j), C.c_void_p), tlens.ctypes.data + 2 * j, m,
                        st.ctypes.data + j, cs.ctypes.data + 4 * j, C.byref(t)))
                    j += m
                assert t.value != 0
                tickets.append(t.value)
                if len(tickets) % 13 == 0:
                    gpucsum.check(L.gcs_wait(c.h, tickets[-9]))
            gpucsum.check(L.gcs_wait(c.h, tickets[-1]))
    finally:
        if registered:
            gpucsum.check(L.gcs_host_unregister(mem.ctypes.data + base))
    np.testing.assert_array_equal(vd, rv)
    assert (vd[bad] != 0).all()
    np.testing.assert_array_equal(rxm, rref)              # the side effect, exactly
    np.testing.assert_array_equal(st, rst)
    np.testing.assert_array_equal(cs, rcs)
    np.testing.assert_array_equal(txm, tref)


def test_async_fill_without_server_is_synchronous(torch_dev):
    import ctypes as C
    L = gpucsum.lib()
    L.gcs_compute_ptrs_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
    buf, off, lens = synth.packed_frames(synth.imix_lengths(64, seed=71), seed=72)
    ref = buf.copy()
    rst, _ = Oracle().compute_batch(ref, off, lens)
    ptrs = (C.c_void_p * len(off))(*[buf.ctypes.data + int(o) for o in off])
    st = np.zeros(len(off), np.uint8)
    t = C.c_uint64(123)
    with gpucsum.Context(0, max_frames=1024, max_bytes=4 << 20) as c:
        gpucsum.check(L.gcs_compute_ptrs_async(c.h, ptrs, lens.ctypes.data, len(off),
                                               st.ctypes.data, None, C.byref(t)))
    assert t.value == 0                     # done on return
    np.testing.assert_array_equal(st, rst)
    np.testing.assert_array_equal(buf, ref)


def test_server_requests_of_every_size_and_mode_over_the_slots(torch_dev):
    """ADVICE r05 (torn request lines): 1,600 async requests on ONE ring -- fills
    and verifies at random, 1..64 frames each, verifies with and without the
    tcp_in.c:1237 side effect -- so every one of the ring's 8 slots is reused
    ~200 times with n and mode changing each time.  A poll that took a line
    half from the slot's previous request would serve the wrong count, the
    wrong kind or the wrong frames; every status, check, verdict and frame
    must equal the oracle's."""
    import ctypes as C
    L = gpucsum.lib()
    L.gcs_verify_ptrs_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                        C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
    L.gcs_compute_ptrs_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
    L.gcs_wait.argtypes = [C.c_void_p, C.c_uint64]
    O = Oracle()
    rng = np.random.default_rng(2606)
    reqs = 1600
    sizes = rng.integers(1, 65, size=reqs)
    kinds = rng.integers(0, 3, size=reqs)          # 0 fill, 1 verify, 2 verify + side effect
    n = int(sizes.sum())
    buf, off, lens = synth.packed_frames(synth.imix_lengths(n, seed=2607), seed=2608)
    is_rx = np.repeat(kinds != 0, sizes)
    rx_idx = np.nonzero(is_rx)[0]
    O.compute_batch(buf, off[rx_idx], lens[rx_idx])   # RX frames carry valid checks ...
    synth.corrupt(buf, off[rx_idx], lens[rx_idx], frac_log2=3, seed=2609)   # ... some broken
    ref = buf.copy()
    exp_code = np.zeros(n, np.uint8)
    exp_cs = np.zeros(n, np.uint32)
    i = 0
    for m, k in zip(sizes, kinds):
        sl = slice(i, i + int(m))
        if k == 0:
            exp_code[sl], exp_cs[sl] = O.compute_batch(ref, off[sl], lens[sl])
        else:
            exp_code[sl] = O.verify_batch(ref, off[sl], lens[sl], flags=1 if k == 2 else 0)
        i += int(m)
    ptrs = (C.c_void_p * n)(*[buf.ctypes.data + int(o) for o in off])
    code = np.full(n, 0xEE, np.uint8)
    cs = np.zeros(n, np.uint32)
    with gpucsum.Context(0, max_frames=4096, max_bytes=8 << 20) as c:
        c.set_burst_server(True)
        tickets = []
        i = 0
        for r, (m, k) in enumerate(zip(sizes, kinds)):
            m = int(m)
            t = C.c_uint64()
            p = C.cast(C.byref(ptrs, 8 * i), C.c_void_p)
            if k == 0:
                gpucsum.check(L.gcs_compute_ptrs_async(c.h, p, lens.ctypes.data + 2 * i, m,
                                                       code.ctypes.data + i, cs.ctypes.data + 4 * i,
                                                       C.byref(t)))
            else:
                gpucsum.check(L.gcs_verify_ptrs_async(c.h, p, lens.ctypes.data + 2 * i, m,
                                                      code.ctypes.data + i, 1 if k == 2 else 0,
                                                      C.byref(t)))
            assert t.value != 0
            tickets.append(t.value)
            i += m
            if r % 37 == 36:
                gpucsum.check(L.gcs_wait(c.h, tickets[-int(rng.integers(1, 9))]))
        gpucsum.check(L.gcs_wait(c.h, tickets[-1]))
    np.testing.assert_array_equal(code, exp_code)
    tx = ~is_rx
    np.testing.assert_array_equal(cs[tx], exp_cs[tx])
    np.testing.assert_array_equal(buf, ref)


def test_failed_wait_reports_later_requests_to_their_own_wait(torch_dev, monkeypatch):
    """A failed gcs_wait reports the cancelled fills up to its ticket; fills
    posted after that ticket stay cancelled and fail their OWN wait once
    (GCS_EHIP: their outputs were never written), then read as done; a
    cancelled verify is reported once to the first verify wait covering it.
    Nothing reports success for results it never produced."""
    import ctypes as C
    L = gpucsum.lib()
    L.gcs_compute_ptrs_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
    L.gcs_verify_ptrs_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                        C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
    L.gcs_wait.argtypes = [C.c_void_p, C.c_uint64]
    EHIP = gpucsum.K["GCS_EHIP"]
    monkeypatch.setenv("GCS_FAULT_INJECT", "none")        # arms the context's fault hooks
    buf, off, lens = synth.packed_frames(synth.imix_lengths(80, seed=171), seed=172)
    ptrs = (C.c_void_p * len(off))(*[buf.ctypes.data + int(o) for o in off])
    st = np.zeros(len(off), np.uint8)
    vd = np.zeros(len(off), np.uint8)
    with gpucsum.Context(0, max_frames=1024, max_bytes=4 << 20) as c:
        c.set_burst_server(True)
        tk = []
        for k in range(5):                    # fills f0..f3 and one verify (k = 2)
            t = C.c_uint64()
            p = C.cast(C.byref(ptrs, 8 * 16 * k), C.c_void_p)
            if k == 2:
                gpucsum.check(L.gcs_verify_ptrs_async(c.h, p, lens.ctypes.data + 32 * k, 16,
                                                      vd.ctypes.data + 16 * k, 0, C.byref(t)))
            else:
                gpucsum.check(L.gcs_compute_ptrs_async(c.h, p, lens.ctypes.data + 32 * k, 16,
                                                       st.ctypes.data + 16 * k, None,
                                                       C.byref(t)))
            assert t.value != 0
            tk.append(t.value)
        monkeypatch.setenv("GCS_FAULT_INJECT", "wait")
        assert L.gcs_wait(c.h, tk[1]) == EHIP          # reports f0, f1
        monkeypatch.setenv("GCS_FAULT_INJECT", "none")
        assert L.gcs_wait(c.h, tk[3]) == EHIP          # f2 (k = 3): its own wait
        assert L.gcs_wait(c.h, tk[4]) == EHIP          # f3 (k = 4): its own wait
        assert L.gcs_wait(c.h, tk[4]) == 0             # reported once
        assert L.gcs_wait(c.h, tk[2]) == EHIP          # the verify, to a verify wait
        assert L.gcs_wait(c.h, tk[2]) == 0
        # the ring serves on: a fresh fill completes exactly
        ref = buf.copy()
        rst, _ = Oracle().compute_batch(ref, off, lens)
        t = C.c_uint64()
        gpucsum.check(L.gcs_compute_ptrs_async(c.h, ptrs, lens.ctypes.data, 16, st.ctypes.data,
                                               None, C.byref(t)))
        gpucsum.check(L.gcs_wait(c.h, t.value))
        np.testing.assert_array_equal(st[:16], rst[:16])


@pytest.mark.parametrize("life_us", [2000, 150])
def test_hub_serves_many_contexts_at_once(torch_dev, monkeypatch, life_us):
    """One grid per process serves the rings of 12 contexts, one per thread,
    posting at once (mTCP threads on one GPU); contexts join while the grid
    serves the others (each join makes it leave and restart), and with a
    150 us lifetime the grid also leaves mid-traffic and a fresh one resumes
    every ring where each block stopped.  Every burst equals the oracle."""
    import threading
    monkeypatch.setenv("GCS_SERVER_LIFE_US", str(life_us))
    O = Oracle()
    errors = []

    def worker(w):
        try:
            with gpucsum.Context(0, max_frames=1024, max_bytes=4 << 20) as c:
                c.set_burst_server(True)
                for k, (buf, off, lens) in enumerate(bursts(12, 64, 1000 + 37 * w)):
                    b1 = buf.copy()
                    st, cs = c.compute_host(b1, off, lens)
                    ref = buf.copy()
                    rst, rcs = O.compute_batch(ref, off, lens)
                    np.testing.assert_array_equal(st, rst)
                    np.testing.assert_array_equal(cs, rcs)
                    np.testing.assert_array_equal(b1, ref)
                    bad = synth.corrupt(ref, off, lens, frac_log2=2, seed=k + w)
                    v = c.verify_host(ref.copy(), off, lens)
                    np.testing.assert_array_equal(v, O.verify_batch(ref.copy(), off, lens))
                    assert (v[bad] != 0).all()
        except Exception as e:                 # noqa: BLE001 (re-raised below)
            errors.append((w, e))

    th = [threading.Thread(target=worker, args=(w,)) for w in range(12)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not any(t.is_alive() for t in th)
    assert not errors, errors[:2]


HUB_RINGS = 32   # gcs_internal.h kHubRings: contexts one device's grid serves


def test_hub_ring_limit(torch_dev):
    """A 33rd context of the process gets GCS_ERANGE from
    gcs_ctx_set_burst_server and still serves its bursts (launch per batch);
    every one of the 32 rings serves its own; a ring freed by a leaving
    context is taken again."""
    L = gpucsum.lib()
    O = Oracle()
    ctxs = [gpucsum.Context(0, max_frames=256, max_bytes=1 << 20) for _ in range(HUB_RINGS + 1)]
    try:
        for c in ctxs[:HUB_RINGS]:
            c.set_burst_server(True)
        assert L.gcs_ctx_set_burst_server(ctxs[HUB_RINGS].h, 1) == gpucsum.K["GCS_ERANGE"]
        for j, c in enumerate(ctxs):
            buf, off, lens = bursts(1, 64, 1300 + j)[0]
            v = c.verify_host(buf.copy(), off, lens)
            np.testing.assert_array_equal(v, O.verify_batch(buf.copy(), off, lens))
        ctxs[3].set_burst_server(False)
        gpucsum.check(L.gcs_ctx_set_burst_server(ctxs[HUB_RINGS].h, 1))
        buf, off, lens = bursts(1, 64, 1400)[0]
        v = ctxs[HUB_RINGS].verify_host(buf.copy(), off, lens)
        np.testing.assert_array_equal(v, O.verify_batch(buf.copy(), off, lens))
    finally:
        for c in ctxs:
            c.close()


def test_hub_grid_holds_no_launch_back(torch_dev, monkeypatch):
    """The resident grid runs on a highest-priority stream of its own: while
    it stays resident (idle and lifetime exits set to 5 s), another context's
    launches -- a DMA batch too large for the server -- finish in well under
    the grid's lifetime instead of queueing behind it."""
    import time
    monkeypatch.setenv("GCS_SERVER_IDLE_US", "5000000")
    monkeypatch.setenv("GCS_SERVER_LIFE_US", "5000000")
    O = Oracle()
    big = bursts(1, 20000, 1500)[0]
    with gpucsum.Context(0, max_frames=1024, max_bytes=4 << 20) as cs, \
            gpucsum.Context(0, max_frames=1 << 15, max_bytes=32 << 20) as cb:
        cs.set_burst_server(True)
        buf, off, lens = bursts(1, 64, 1501)[0]
        np.testing.assert_array_equal(cs.verify_host(buf.copy(), off, lens),
                                      O.verify_batch(buf.copy(), off, lens))
        buf, off, lens = big
        cb.verify_host(buf.copy(), off, lens)          # warm-up (first launches)
        t0 = time.perf_counter()
        v = cb.verify_host(buf.copy(), off, lens)
        dt = time.perf_counter() - t0
        np.testing.assert_array_equal(v, O.verify_batch(buf.copy(), off, lens))
        assert dt < 0.5, dt
        # and the grid still serves
        buf, off, lens = bursts(1, 64, 1502)[0]
        np.testing.assert_array_equal(cs.verify_host(buf.copy(), off, lens),
                                      O.verify_batch(buf.copy(), off, lens))
