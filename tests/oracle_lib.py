"""ctypes bindings for the CPU checkers under oracle/ (test infrastructure).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product (mtcp_amd/, libmtcp_gpucsum.so) never does.

* ``Oracle``    -> oracle/liboracle_csum.so   (clean-room restatement)
* ``RefHarness``-> oracle/_ref/libref_mtcp_csum.so (the reference's own
  TCPCalcChecksum + ip_fast_csum, built from /root/reference by
  oracle/Makefile; absent on a box where it was never built)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle_csum.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libref_mtcp_csum.so")

_u8p = C.POINTER(C.c_uint8)


def _p(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


def build_oracle() -> None:
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", ORACLE_DIR, "all"], check=True,
                       stdout=subprocess.DEVNULL)


class Oracle:
    def __init__(self):
        build_oracle()
        L = C.CDLL(ORACLE_SO)
        L.ref_tcp_calc_checksum.restype = C.c_uint16
        L.ref_tcp_calc_checksum.argtypes = [C.c_void_p, C.c_uint16, C.c_uint32, C.c_uint32]
        L.ref_ip_fast_csum.restype = C.c_uint16
        L.ref_ip_fast_csum.argtypes = [C.c_void_p, C.c_uint]
        L.ref_rx_verdict.restype = C.c_int
        L.ref_rx_verdict.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.ref_tx_fill.restype = C.c_int
        L.ref_tx_fill.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.ref_verify_batch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                       C.c_uint32, C.c_void_p, C.c_uint32]
        L.ref_compute_batch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                        C.c_uint32, C.c_void_p, C.c_void_p]
        L.ref_verify_fixed.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                       C.c_void_p, C.c_uint32]
        L.ref_compute_fixed.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                        C.c_void_p, C.c_void_p]
        L.ref_verify_fixed_mt.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                          C.c_void_p, C.c_uint32, C.c_int]
        L.ref_compute_fixed_mt.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                           C.c_void_p, C.c_void_p, C.c_int]
        L.ref_tcp_checksum_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_void_p, C.c_uint32, C.c_void_p]
        L.ref_ip_checksum_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                            C.c_void_p]
        L.ref_icmp_checksum.restype = C.c_uint16
        L.ref_icmp_checksum.argtypes = [C.c_void_p, C.c_int]
        L.ref_icmp_checksum_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                              C.c_void_p]
        L.ref_tx_fill_f.restype = C.c_int
        L.ref_tx_fill_f.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
        L.ref_compute_batch_f.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                          C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32]
        L.ref_compute_copy_batch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                             C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p,
                                             C.c_void_p, C.c_void_p]
        L.ref_gro_batch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64,
                                    C.c_void_p, C.c_void_p, C.c_void_p]
        L.ref_rss_hash.restype = C.c_uint32
        L.ref_rss_hash.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16]
        L.ref_rss_core.restype = C.c_int
        L.ref_rss_core.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16,
                                   C.c_int, C.c_int]
        L.ref_classify_batch.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                         C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_uint32, C.c_void_p, C.c_int, C.c_int]
        L.ref_classify_fixed.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.c_void_p, C.c_int, C.c_int]
        self.L = L

    # -- element functions -------------------------------------------------
    def tcp_calc_checksum(self, buf: bytes, length: int, saddr: int, daddr: int) -> int:
        b = np.frombuffer(bytes(buf) + b"\0\0", dtype=np.uint8).copy()
        return self.L.ref_tcp_calc_checksum(_p(b), length, saddr, daddr)

    def ip_fast_csum(self, hdr: bytes, ihl: int) -> int:
        b = np.frombuffer(bytes(hdr) + b"\0" * 64, dtype=np.uint8).copy()
        return self.L.ref_ip_fast_csum(_p(b), ihl)

    def icmp_checksum(self, buf: bytes, length: int) -> int:
        b = np.frombuffer(bytes(buf) + b"\0\0", dtype=np.uint8).copy()
        return self.L.ref_icmp_checksum(_p(b), length)

    @staticmethod
    def _key(key):
        if key is None:
            return None
        k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
        assert k.size >= 16
        return k

    def rss_hash(self, sip, dip, sp, dp, key=None) -> int:
        k = self._key(key)
        return self.L.ref_rss_hash(_p(k), sip, dip, sp, dp)

    def rss_core(self, sip, dip, sp, dp, num_queues, endian_check, key=None) -> int:
        k = self._key(key)
        return self.L.ref_rss_core(_p(k), sip, dip, sp, dp, num_queues, endian_check)

    # -- batches ----------------------------------------------------------
    def classify_batch(self, buf, off, lens, num_queues, endian_check, key=None, flags=0):
        n = len(off)
        vd = np.zeros(n, dtype=np.uint8)
        h = np.zeros(n, dtype=np.uint32)
        q = np.zeros(n, dtype=np.uint16)
        k = self._key(key)
        self.L.ref_classify_batch(_p(buf), buf.nbytes, _p(np.ascontiguousarray(off, np.uint64)),
                                  _p(np.ascontiguousarray(lens, np.uint16)), n, _p(vd), _p(h),
                                  _p(q), flags, _p(k), num_queues, endian_check)
        return vd, h, q

    def classify_fixed(self, buf, stride, frame_len, n, num_queues, endian_check, key=None,
                       flags=0):
        vd = np.zeros(n, dtype=np.uint8)
        h = np.zeros(n, dtype=np.uint32)
        q = np.zeros(n, dtype=np.uint16)
        k = self._key(key)
        self.L.ref_classify_fixed(_p(buf), stride, frame_len, n, _p(vd), _p(h), _p(q), flags,
                                  _p(k), num_queues, endian_check)
        return vd, h, q

    def compute_copy_batch(self, buf, off, lens, src, src_off):
        n = len(off)
        st = np.zeros(n, dtype=np.uint8)
        cs = np.zeros(n, dtype=np.uint32)
        self.L.ref_compute_copy_batch(_p(buf), buf.nbytes,
                                      _p(np.ascontiguousarray(off, np.uint64)),
                                      _p(np.ascontiguousarray(lens, np.uint16)), n, _p(src),
                                      src.nbytes, _p(np.ascontiguousarray(src_off, np.uint64)),
                                      _p(st), _p(cs))
        return st, cs

    def gro_batch(self, buf, off, lens, verdict, window, max_len, out_bytes=None):
        """-> (out buffer, out_off, out_len, head)"""
        n = len(off)
        out = np.zeros(buf.nbytes if out_bytes is None else out_bytes, dtype=np.uint8)
        oo = np.zeros(n, dtype=np.uint64)
        ol = np.zeros(n, dtype=np.uint16)
        hd = np.zeros(n, dtype=np.uint32)
        self.L.ref_gro_batch(_p(buf), buf.nbytes, _p(np.ascontiguousarray(off, np.uint64)),
                             _p(np.ascontiguousarray(lens, np.uint16)),
                             _p(np.ascontiguousarray(verdict, np.uint8)), n, window, max_len,
                             _p(out), out.nbytes, _p(oo), _p(ol), _p(hd))
        return out, oo, ol, hd

    def icmp_checksum_batch(self, buf, off, lens):
        n = len(off)
        out = np.zeros(n, dtype=np.uint16)
        self.L.ref_icmp_checksum_batch(_p(buf), _p(np.ascontiguousarray(off, np.uint64)),
                                       _p(np.ascontiguousarray(lens, np.uint16)), n, _p(out))
        return out

    def verify_batch(self, buf, off, lens, flags=0):
        n = len(off)
        out = np.zeros(n, dtype=np.uint8)
        self.L.ref_verify_batch(_p(buf), buf.nbytes, _p(np.ascontiguousarray(off, np.uint64)),
                                _p(np.ascontiguousarray(lens, np.uint16)), n, _p(out), flags)
        return out

    def compute_batch(self, buf, off, lens, flags=0):
        n = len(off)
        st = np.zeros(n, dtype=np.uint8)
        cs = np.zeros(n, dtype=np.uint32)
        self.L.ref_compute_batch_f(_p(buf), buf.nbytes,
                                   _p(np.ascontiguousarray(off, np.uint64)),
                                   _p(np.ascontiguousarray(lens, np.uint16)), n, _p(st), _p(cs),
                                   flags)
        return st, cs

    def verify_fixed(self, buf, stride, frame_len, n, flags=0, threads=1):
        out = np.zeros(n, dtype=np.uint8)
        if threads == 1:
            self.L.ref_verify_fixed(_p(buf), stride, frame_len, n, _p(out), flags)
        else:
            self.L.ref_verify_fixed_mt(_p(buf), stride, frame_len, n, _p(out), flags, threads)
        return out

    def compute_fixed(self, buf, stride, frame_len, n, threads=1, want=True):
        st = np.zeros(n, dtype=np.uint8) if want else None
        cs = np.zeros(n, dtype=np.uint32) if want else None
        if threads == 1:
            self.L.ref_compute_fixed(_p(buf), stride, frame_len, n, _p(st), _p(cs))
        else:
            self.L.ref_compute_fixed_mt(_p(buf), stride, frame_len, n, _p(st), _p(cs), threads)
        return st, cs

    def tcp_checksum_batch(self, buf, off, lens, saddr, daddr):
        n = len(off)
        out = np.zeros(n, dtype=np.uint16)
        self.L.ref_tcp_checksum_batch(_p(buf), _p(np.ascontiguousarray(off, np.uint64)),
                                      _p(np.ascontiguousarray(lens, np.uint16)),
                                      _p(np.ascontiguousarray(saddr, np.uint32)),
                                      _p(np.ascontiguousarray(daddr, np.uint32)), n, _p(out))
        return out

    def ip_checksum_batch(self, buf, off, ihl):
        n = len(off)
        out = np.zeros(n, dtype=np.uint16)
        self.L.ref_ip_checksum_batch(_p(buf), _p(np.ascontiguousarray(off, np.uint64)),
                                     _p(np.ascontiguousarray(ihl, np.uint8)), n, _p(out))
        return out


class RefHarness:
    """The reference's own fold code (oracle/_ref).  ``available()`` is False
    where it was never built (e.g. a GPU box fed a snapshot without it)."""

    @staticmethod
    def available() -> bool:
        return os.path.exists(REF_SO)

    def __init__(self):
        L = C.CDLL(REF_SO)
        L.refx_tcp_calc_checksum.restype = C.c_uint16
        L.refx_tcp_calc_checksum.argtypes = [C.c_void_p, C.c_uint16, C.c_uint32, C.c_uint32]
        L.refx_ip_fast_csum.restype = C.c_uint16
        L.refx_ip_fast_csum.argtypes = [C.c_void_p, C.c_uint]
        L.refx_rx_verdict.restype = C.c_int
        L.refx_rx_verdict.argtypes = [C.c_void_p, C.c_uint32]
        L.refx_tx_fill.restype = C.c_int
        L.refx_tx_fill.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.refx_verify_fixed.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                        C.c_void_p]
        L.refx_compute_fixed.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                         C.c_void_p]
        L.refx_run_fixed_mt.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                        C.c_void_p, C.c_int, C.c_int]
        L.refx_run_fixed_pinned.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                            C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.refx_icmp_checksum.restype = C.c_uint16
        L.refx_icmp_checksum.argtypes = [C.c_void_p, C.c_int]
        L.refx_rss_hash.restype = C.c_uint32
        L.refx_rss_hash.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16]
        L.refx_rss_core.restype = C.c_int
        L.refx_rss_core.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16, C.c_int,
                                    C.c_int]
        L.refx_rx_verdict_f.restype = C.c_int
        L.refx_rx_verdict_f.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.refx_tx_fill_f.restype = C.c_int
        L.refx_tx_fill_f.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
        self.L = L

    def icmp_checksum_at(self, buf: np.ndarray, pos: int, length: int) -> int:
        return self.L.refx_icmp_checksum(C.c_void_p(buf.ctypes.data + pos), length)

    def rss_hash(self, sip: int, dip: int, sp: int, dp: int) -> int:
        return self.L.refx_rss_hash(sip, dip, sp, dp)

    def rss_core(self, sip: int, dip: int, sp: int, dp: int, num_queues: int,
                 endian_check: int) -> int:
        return self.L.refx_rss_core(sip, dip, sp, dp, num_queues, endian_check)

    def rx_verdict_f_at(self, buf: np.ndarray, pos: int, length: int, flags: int) -> int:
        return self.L.refx_rx_verdict_f(C.c_void_p(buf.ctypes.data + pos), length, flags)

    def tx_fill_f_at(self, buf: np.ndarray, pos: int, length: int,
                     flags: int) -> tuple[int, int]:
        cs = C.c_uint32(0)
        st = self.L.refx_tx_fill_f(C.c_void_p(buf.ctypes.data + pos), length, C.byref(cs), flags)
        return st, cs.value

    def tcp_calc_checksum_at(self, buf: np.ndarray, pos: int, length: int, saddr: int,
                             daddr: int) -> int:
        return self.L.refx_tcp_calc_checksum(C.c_void_p(buf.ctypes.data + pos), length,
                                             saddr, daddr)

    def ip_fast_csum_at(self, buf: np.ndarray, pos: int, ihl: int) -> int:
        return self.L.refx_ip_fast_csum(C.c_void_p(buf.ctypes.data + pos), ihl)

    def rx_verdict_at(self, buf: np.ndarray, pos: int, length: int) -> int:
        return self.L.refx_rx_verdict(C.c_void_p(buf.ctypes.data + pos), length)

    def tx_fill_at(self, buf: np.ndarray, pos: int, length: int) -> tuple[int, int]:
        cs = C.c_uint32(0)
        st = self.L.refx_tx_fill(C.c_void_p(buf.ctypes.data + pos), length, C.byref(cs))
        return st, cs.value

    def run_fixed(self, buf, stride, frame_len, n, compute, threads=1, cpus=None):
        """cpus: pin thread t to cpus[t] (len(cpus) threads); None: unpinned."""
        out = np.zeros(n, dtype=np.uint8)
        if cpus is None:
            self.L.refx_run_fixed_mt(_p(buf), stride, frame_len, n, _p(out), int(compute),
                                     threads)
            return out
        c = np.ascontiguousarray(cpus, np.int32)
        assert self.L.refx_run_fixed_pinned(_p(buf), stride, frame_len, n, _p(out),
                                            int(compute), len(c), _p(c)) == 0
        return out
