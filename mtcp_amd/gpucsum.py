"""ctypes binding of libmtcp_gpucsum.so (include/mtcp_gpucsum.h).

This is plumbing for tests and bench.py: every call goes straight into the
HIP C ABI.  There is no CPU fallback -- if the library or a GPU is missing,
construction raises.

Device buffers may be given as torch tensors (``.data_ptr()`` is used) or as
raw integer addresses; host buffers as numpy arrays.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "lib", "libmtcp_gpucsum.so")
HEADER = os.path.join(ROOT, "include", "mtcp_gpucsum.h")


def _constants() -> dict[str, int]:
    """GCS_* integer macros parsed from the public header (single source)."""
    out = {}
    for m in re.finditer(r"#define\s+(GCS_[A-Z0-9_]+)\s+\(?(-?(?:0x)?[0-9a-fA-F]+)u?\)?",
                         open(HEADER).read()):
        out[m.group(1)] = int(m.group(2), 0)
    return out


K = _constants()
V_NAMES = {v: k[6:] for k, v in K.items() if k.startswith("GCS_V_") and k != "GCS_V_IS_ERROR"}


class GcsError(RuntimeError):
    def __init__(self, msg: str, code: int | None = None):
        super().__init__(msg)
        self.code = code


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GcsError(f"{LIB_PATH} is missing: build it with `make -C mtcp_amd/csrc` "
                           "(there is no CPU fallback)")
        # One HIP runtime per process.  PyTorch-ROCm bundles its own
        # libamdhip64 / libhsa-runtime64; if this library were loaded first it
        # would bring in /opt/rocm's copies and torch would then load its own,
        # a second HSA runtime instance in the process, one of which sees no
        # device ("no ROCm-capable device").  Loading torch first makes our
        # libamdhip64.so.7 dependency resolve to torch's already-loaded copy.
        # (A C program such as mTCP has no torch: /opt/rocm's runtime alone.)
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        vp, u8, u16, u32, u64, i = (C.c_void_p, C.c_uint8, C.c_uint16, C.c_uint32, C.c_uint64,
                                    C.c_int)
        sig = {
            "gcs_abi_version": (i, []),
            "gcs_strerror": (C.c_char_p, [i]),
            "gcs_last_hip_error": (C.c_char_p, []),
            "gcs_device_count": (i, [C.POINTER(i)]),
            "gcs_ctx_create": (i, [C.POINTER(vp), i, u32, u64]),
            "gcs_ctx_destroy": (i, [vp]),
            "gcs_ctx_device": (i, [vp, C.POINTER(i)]),
            "gcs_ctx_stream": (i, [vp, C.POINTER(vp)]),
            "gcs_sync": (i, [vp]),
            "gcs_device_check": (i, [i]),
            "gcs_host_alloc": (i, [C.POINTER(vp), u64]),
            "gcs_host_free": (i, [vp]),
            "gcs_host_register": (i, [vp, u64]),
            "gcs_host_unregister": (i, [vp]),
            "gcs_dev_alloc": (i, [vp, C.POINTER(vp), u64]),
            "gcs_dev_free": (i, [vp, vp]),
            "gcs_verify_fixed_dev": (i, [vp, vp, u64, u32, u32, vp, u32, vp]),
            "gcs_compute_fixed_dev": (i, [vp, vp, u64, u32, u32, vp, vp, u32, vp]),
            "gcs_step_fixed_dev": (i, [vp, vp, u64, u32, u32, vp, vp, u32, vp, u64, u32, u32,
                                       vp, u32, vp]),
            "gcs_verify_dev": (i, [vp, vp, u64, vp, vp, u32, vp, u32, vp]),
            "gcs_compute_dev": (i, [vp, vp, u64, vp, vp, u32, vp, vp, u32, vp]),
            "gcs_tcp_checksum_dev": (i, [vp, vp, u64, vp, vp, vp, vp, u32, vp, vp]),
            "gcs_ip_checksum_dev": (i, [vp, vp, u64, vp, vp, u32, vp, vp]),
            "gcs_verify": (i, [vp, vp, vp, vp, u32, vp, u32]),
            "gcs_compute": (i, [vp, vp, vp, vp, u32, vp, vp]),
            "gcs_verify_ptrs": (i, [vp, vp, vp, u32, vp, u32]),
            "gcs_compute_ptrs": (i, [vp, vp, vp, u32, vp, vp]),
            "gcs_icmp_checksum_dev": (i, [vp, vp, u64, vp, vp, u32, vp, vp]),
            "gcs_gro_dev": (i, [vp, vp, u64, vp, vp, vp, u32, u32, u32, vp, u64, vp, vp, vp,
                                vp]),
            "gcs_compute_copy_dev": (i, [vp, vp, u64, vp, vp, vp, u64, vp, u32, vp, vp, u32,
                                         vp]),
            "gcs_ctx_set_rss": (i, [vp, vp, u32, u32, i]),
            "gcs_ctx_set_burst_server": (i, [vp, i]),
            "gcs_classify_fixed_dev": (i, [vp, vp, u64, u32, u32, vp, vp, vp, u32, vp]),
            "gcs_classify_dev": (i, [vp, vp, u64, vp, vp, u32, vp, vp, vp, u32, vp]),
            "gcs_rss_dev": (i, [vp, vp, vp, vp, vp, u32, vp, vp, vp]),
            "gcs_classify": (i, [vp, vp, vp, vp, u32, vp, vp, vp, u32]),
            "gcs_classify_ptrs": (i, [vp, vp, vp, u32, vp, vp, vp, u32]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        del u8, u16
        _lib = L
    return _lib


def _addr(x):
    """Device/host address of a torch tensor, numpy array, int or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        assert x.flags["C_CONTIGUOUS"]
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        assert x.is_contiguous()
        return x.data_ptr()
    raise TypeError(type(x))


def _daddr(x):
    """Address of a DEVICE buffer: a CUDA/HIP torch tensor or a raw int.
    Host arrays are refused (a kernel touching them would fault the GPU)."""
    if x is None or isinstance(x, int):
        return x
    if isinstance(x, np.ndarray) or not getattr(x, "is_cuda", False):
        raise GcsError("device entry point given a host buffer")
    return _addr(x)


def _nbytes(x) -> int:
    if isinstance(x, np.ndarray):
        return x.nbytes
    if hasattr(x, "data_ptr"):
        return x.numel() * x.element_size()
    raise TypeError("pass nbytes explicitly for raw addresses")


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        L = lib()
        raise GcsError(f"{what}: {L.gcs_strerror(rc).decode()} ({rc}) "
                       f"{L.gcs_last_hip_error().decode()}", rc)


def device_check(device: int = 0) -> None:
    """gcs_device_check: every stream drained without a fault and no burst
    server grid resident without a ring; raises GcsError otherwise."""
    check(lib().gcs_device_check(device), "gcs_device_check")


def device_count() -> int:
    c = C.c_int(0)
    rc = lib().gcs_device_count(C.byref(c))
    return c.value if rc == 0 else 0


def _torch_ordered(stream, *bufs):
    """Stream ordering for stream=None launches.  They run on the context's
    own (non-blocking) HIP stream, which does not wait for torch's stream: a
    torch.zeros() / copy still in flight there would race the kernel.  So
    when a torch CUDA tensor is passed without an explicit stream, wait for
    torch's current stream first.  (bench.py passes torch's stream instead.)"""
    if stream is not None:
        return
    for b in bufs:
        if getattr(b, "is_cuda", False):
            import torch
            torch.cuda.current_stream().synchronize()
            return


class Context:
    """One gcs_ctx: a HIP device + stream (+ pinned staging for host batches)."""

    def __init__(self, device: int = 0, max_frames: int = 0, max_bytes: int = 0):
        self.L = lib()
        h = C.c_void_p()
        check(self.L.gcs_ctx_create(C.byref(h), device, max_frames, max_bytes), "gcs_ctx_create")
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            check(self.L.gcs_ctx_destroy(self.h), "gcs_ctx_destroy")
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def stream(self) -> int:
        s = C.c_void_p()
        check(self.L.gcs_ctx_stream(self.h, C.byref(s)))
        return s.value or 0

    def sync(self):
        check(self.L.gcs_sync(self.h), "gcs_sync")

    # -- device-resident batches -------------------------------------------
    @staticmethod
    def _need(buf, nbytes, what):
        """Host-side shape check before a launch: a kernel must never be
        pointed past the end of a buffer (GPU faults take the box down)."""
        if buf is None or isinstance(buf, int):
            return
        if _nbytes(buf) < nbytes:
            raise GcsError(f"{what}: buffer of {_nbytes(buf)} B < required {nbytes} B")

    def verify_fixed(self, frames, stride, frame_len, n, verdict, flags=0, stream=None):
        _torch_ordered(stream, frames, verdict)
        self._need(frames, n * stride, "frames")
        self._need(verdict, n, "verdict")
        check(self.L.gcs_verify_fixed_dev(self.h, _daddr(frames), stride, frame_len, n,
                                          _daddr(verdict), flags, stream), "verify_fixed")

    def compute_fixed(self, frames, stride, frame_len, n, status=None, csums=None, flags=0,
                      stream=None):
        _torch_ordered(stream, frames, status, csums)
        self._need(frames, n * stride, "frames")
        self._need(status, n, "status")
        self._need(csums, 4 * n, "csums")
        check(self.L.gcs_compute_fixed_dev(self.h, _daddr(frames), stride, frame_len, n,
                                           _daddr(status), _daddr(csums), flags, stream),
              "compute_fixed")

    def step_fixed(self, tx, tx_stride, tx_len, n_tx, rx, rx_stride, rx_len, n_rx, verdict,
                   tx_status=None, tx_csums=None, tx_flags=0, rx_flags=0, stream=None):
        """gcs_step_fixed_dev: TX fill of `tx` and RX verify of `rx` in one launch."""
        _torch_ordered(stream, tx, rx, verdict, tx_status, tx_csums)
        self._need(tx, n_tx * tx_stride, "tx")
        self._need(rx, n_rx * rx_stride, "rx")
        self._need(verdict, n_rx, "verdict")
        self._need(tx_status, n_tx, "tx_status")
        self._need(tx_csums, 4 * n_tx, "tx_csums")
        check(self.L.gcs_step_fixed_dev(self.h, _daddr(tx), tx_stride, tx_len, n_tx,
                                        _daddr(tx_status), _daddr(tx_csums), tx_flags, _daddr(rx),
                                        rx_stride, rx_len, n_rx, _daddr(verdict), rx_flags,
                                        stream), "step_fixed")

    def verify(self, frames, off, lens, n, verdict, flags=0, stream=None, frames_bytes=None):
        _torch_ordered(stream, frames, off, lens, verdict)
        fb = _nbytes(frames) if frames_bytes is None else frames_bytes
        self._need(frames, fb, "frames")
        self._need(off, 8 * n, "off")
        self._need(lens, 2 * n, "lens")
        self._need(verdict, n, "verdict")
        check(self.L.gcs_verify_dev(self.h, _daddr(frames), fb, _daddr(off), _daddr(lens), n,
                                    _daddr(verdict), flags, stream), "verify")

    def compute(self, frames, off, lens, n, status=None, csums=None, flags=0, stream=None,
                frames_bytes=None):
        _torch_ordered(stream, frames, off, lens, status, csums)
        fb = _nbytes(frames) if frames_bytes is None else frames_bytes
        self._need(frames, fb, "frames")
        self._need(off, 8 * n, "off")
        self._need(lens, 2 * n, "lens")
        self._need(status, n, "status")
        self._need(csums, 4 * n, "csums")
        check(self.L.gcs_compute_dev(self.h, _daddr(frames), fb, _daddr(off), _daddr(lens), n,
                                     _daddr(status), _daddr(csums), flags, stream), "compute")

    def tcp_checksum(self, buf, off, lens, saddr, daddr, n, out, stream=None, buf_bytes=None):
        _torch_ordered(stream, buf, off, lens, saddr, daddr, out)
        bb = _nbytes(buf) if buf_bytes is None else buf_bytes
        self._need(buf, bb, "buf")
        for a, w in ((off, 8), (lens, 2), (saddr, 4), (daddr, 4), (out, 2)):
            self._need(a, w * n, "array")
        check(self.L.gcs_tcp_checksum_dev(self.h, _daddr(buf), bb, _daddr(off), _daddr(lens),
                                          _daddr(saddr), _daddr(daddr), n, _daddr(out), stream),
              "tcp_checksum")

    def ip_checksum(self, buf, off, ihl, n, out, stream=None, buf_bytes=None):
        _torch_ordered(stream, buf, off, ihl, out)
        bb = _nbytes(buf) if buf_bytes is None else buf_bytes
        self._need(buf, bb, "buf")
        for a, w in ((off, 8), (ihl, 1), (out, 2)):
            self._need(a, w * n, "array")
        check(self.L.gcs_ip_checksum_dev(self.h, _daddr(buf), bb, _daddr(off), _daddr(ihl), n,
                                         _daddr(out), stream), "ip_checksum")

    def compute_copy(self, frames, off, lens, src, src_off, n, status=None, csums=None,
                     flags=0, stream=None, frames_bytes=None, src_bytes=None):
        _torch_ordered(stream, frames, off, lens, src, src_off, status, csums)
        fb = _nbytes(frames) if frames_bytes is None else frames_bytes
        sb = _nbytes(src) if src_bytes is None else src_bytes
        self._need(frames, fb, "frames")
        self._need(src, sb, "src")
        for a, w in ((off, 8), (lens, 2), (src_off, 8), (status, 1), (csums, 4)):
            self._need(a, w * n, "array")
        check(self.L.gcs_compute_copy_dev(self.h, _daddr(frames), fb, _daddr(off), _daddr(lens),
                                          _daddr(src), sb, _daddr(src_off), n, _daddr(status),
                                          _daddr(csums), flags, stream), "compute_copy")

    def gro(self, frames, off, lens, verdict, n, window, max_len, out, out_off, out_len, head,
            stream=None, in_bytes=None, out_bytes=None):
        _torch_ordered(stream, frames, off, lens, verdict, out, out_off, out_len, head)
        ib = _nbytes(frames) if in_bytes is None else in_bytes
        ob = _nbytes(out) if out_bytes is None else out_bytes
        self._need(frames, ib, "frames")
        self._need(out, ob, "out")
        for a, w in ((off, 8), (lens, 2), (verdict, 1), (out_off, 8), (out_len, 2), (head, 4)):
            self._need(a, w * n, "array")
        check(self.L.gcs_gro_dev(self.h, _daddr(frames), ib, _daddr(off), _daddr(lens),
                                 _daddr(verdict), n, window, max_len, _daddr(out), ob,
                                 _daddr(out_off), _daddr(out_len), _daddr(head), stream), "gro")

    def icmp_checksum(self, buf, off, lens, n, out, stream=None, buf_bytes=None):
        _torch_ordered(stream, buf, off, lens, out)
        bb = _nbytes(buf) if buf_bytes is None else buf_bytes
        self._need(buf, bb, "buf")
        for a, w in ((off, 8), (lens, 2), (out, 2)):
            self._need(a, w * n, "array")
        check(self.L.gcs_icmp_checksum_dev(self.h, _daddr(buf), bb, _daddr(off), _daddr(lens), n,
                                           _daddr(out), stream), "icmp_checksum")

    # -- RSS steering (rss.c) -------------------------------------------------
    def set_burst_server(self, on: bool = True):
        check(self.L.gcs_ctx_set_burst_server(self.h, 1 if on else 0), "gcs_ctx_set_burst_server")

    def set_rss(self, key: bytes | None = None, num_queues: int = 1, endian_check: int = 0):
        k = None if key is None else np.frombuffer(bytes(key), dtype=np.uint8).copy()
        check(self.L.gcs_ctx_set_rss(self.h, _addr(k), 0 if k is None else k.size, num_queues,
                                     endian_check), "gcs_ctx_set_rss")

    def classify_fixed(self, frames, stride, frame_len, n, verdict, hash=None, queue=None,
                       flags=0, stream=None):
        _torch_ordered(stream, frames, verdict, hash, queue)
        self._need(frames, n * stride, "frames")
        self._need(verdict, n, "verdict")
        self._need(hash, 4 * n, "hash")
        self._need(queue, 2 * n, "queue")
        check(self.L.gcs_classify_fixed_dev(self.h, _daddr(frames), stride, frame_len, n,
                                            _daddr(verdict), _daddr(hash), _daddr(queue), flags,
                                            stream), "classify_fixed")

    def classify(self, frames, off, lens, n, verdict, hash=None, queue=None, flags=0,
                 stream=None, frames_bytes=None):
        _torch_ordered(stream, frames, off, lens, verdict, hash, queue)
        fb = _nbytes(frames) if frames_bytes is None else frames_bytes
        self._need(frames, fb, "frames")
        self._need(off, 8 * n, "off")
        self._need(lens, 2 * n, "lens")
        self._need(verdict, n, "verdict")
        self._need(hash, 4 * n, "hash")
        self._need(queue, 2 * n, "queue")
        check(self.L.gcs_classify_dev(self.h, _daddr(frames), fb, _daddr(off), _daddr(lens), n,
                                      _daddr(verdict), _daddr(hash), _daddr(queue), flags,
                                      stream), "classify")

    def rss(self, sip, dip, sp, dp, n, hash=None, queue=None, stream=None):
        _torch_ordered(stream, sip, dip, sp, dp, hash, queue)
        for a, w in ((sip, 4), (dip, 4), (sp, 2), (dp, 2), (hash, 4), (queue, 2)):
            self._need(a, w * n, "array")
        check(self.L.gcs_rss_dev(self.h, _daddr(sip), _daddr(dip), _daddr(sp), _daddr(dp), n,
                                 _daddr(hash), _daddr(queue), stream), "rss")

    # -- host-memory batches (synchronous) ----------------------------------
    def classify_host(self, frames: np.ndarray, off: np.ndarray, lens: np.ndarray,
                      flags: int = 0):
        n = len(off)
        vd = np.zeros(n, dtype=np.uint8)
        h = np.zeros(n, dtype=np.uint32)
        q = np.zeros(n, dtype=np.uint16)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        check(self.L.gcs_classify(self.h, _addr(frames), _addr(off), _addr(lens), n, _addr(vd),
                                  _addr(h), _addr(q), flags), "gcs_classify")
        return vd, h, q

    def verify_host(self, frames: np.ndarray, off: np.ndarray, lens: np.ndarray,
                    flags: int = 0) -> np.ndarray:
        n = len(off)
        out = np.zeros(n, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        check(self.L.gcs_verify(self.h, _addr(frames), _addr(off), _addr(lens), n, _addr(out),
                                flags), "gcs_verify")
        return out

    def compute_host(self, frames: np.ndarray, off: np.ndarray, lens: np.ndarray):
        n = len(off)
        st = np.zeros(n, dtype=np.uint8)
        cs = np.zeros(n, dtype=np.uint32)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        check(self.L.gcs_compute(self.h, _addr(frames), _addr(off), _addr(lens), n, _addr(st),
                                 _addr(cs)), "gcs_compute")
        return st, cs


class PinnedBuffer:
    """hipHostMalloc'd host memory exposed as a numpy uint8 array."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(lib().gcs_host_alloc(C.byref(p), nbytes), "gcs_host_alloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            self.array = None
            check(lib().gcs_host_free(self.ptr), "gcs_host_free")
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
