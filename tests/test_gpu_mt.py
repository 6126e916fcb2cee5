"""Several mTCP-like threads on ONE GPU at once (tests/plugin/mt_bursts.c).

mTCP maps thread k to GPU k mod n_gpus (gpucsum_module.c), so a 64-core host
with 8 GPUs puts 8 threads -- 8 contexts, with the burst server 8 rings of
the process's one resident grid -- on each device, with HIP's default 4
hardware queues.  Each thread fills and verifies its own 64-frame bursts and
checks every frame against the oracle; all must be exact, and no thread may
stall.
"""
import ctypes as C
import os

import pytest

from mtcp_amd import gpucsum

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MT = os.path.join(ROOT, "tests", "plugin", "libmt_bursts.so")


@pytest.fixture(scope="module")
def M():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (no CPU fallback exists)")
    gpucsum.lib()                      # torch's HIP runtime first, then ours
    L = C.CDLL(MT)
    L.mt_bursts.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint64),
                            C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
    return L


@pytest.mark.parametrize("threads,server", [(1, 1), (1, 0), (4, 1), (4, 0), (8, 1), (8, 0),
                                            (12, 1), (16, 1), (24, 1), (34, 1)])
def test_threads_share_one_gpu(M, threads, server):
    mis, frames, us = C.c_uint64(), C.c_uint64(), C.c_double()
    rc = M.mt_bursts(threads, 200, server, C.byref(mis), C.byref(frames), C.byref(us))
    assert rc == 0, gpucsum.lib().gcs_last_hip_error()
    assert frames.value == threads * 200 * 128
    assert mis.value == 0
    print(f"{threads} threads, server {server}: {us.value:.1f} us per 64-frame call")
    # (34 threads: 32 share the device's grid, the 33rd and 34th launch per
    # call -- gcs_ctx_set_burst_server answers GCS_ERANGE -- and stay exact)
