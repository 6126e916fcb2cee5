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
