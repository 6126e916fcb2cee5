"""How long the RX path keeps the mTCP thread inside the I/O module per burst,
with the plugin verifying each burst as one batch (GPUCSUM_RX_GROUP=0) or as
you go (groups of 8 / 16 / 32 / 64 frames posted in recv_pkts; get_rptr(i)
waits only for frame i's group), through the reference's OWN RX code:
oracle/_ref/libref_mtcp_stack.so's refs_rx_loop_timed, core.c's loop around
mTCP's ProcessPacket (eth_in.c, ip_in.c, tcp_in.c; accepted segments stop at
StreamHTSearch).  The synthetic NIC's RX rooms (2 KiB each, as mbufs) sit in pageable memory (staged by
the library into pinned or, GCS_ASYNC_STAGE=device, device memory) or are
registered with gcs_host_register, as an mbuf pool would be (read in place).  The software path -- the module alone,
mTCP folding every frame on the CPU -- is timed the same way, over pageable
and over registered rooms (software_path_registered).  Prints one JSON
object (tools/, not product)."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (one HIP runtime per process: torch first)
from mtcp_amd import gpucsum, synth  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

vp, u32 = C.c_void_p, C.c_uint32
P = gpucsum.lib()
H = C.CDLL(os.path.join(ROOT, "tests", "plugin", "libplugin_harness.so"))
R = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_mtcp_stack.so"))
H.synth_reset.argtypes = [u32]
H.synth_set_rx.argtypes = [vp, vp, vp, u32]
H.mini_start.argtypes = [vp, vp]
H.mini_stop.argtypes = [vp, vp]
H.synth_rx_base.argtypes = [C.POINTER(C.c_uint64)]
H.synth_rx_base.restype = vp
R.refs_config.argtypes = [u32]
R.refs_rx_loop_timed.argtypes = [vp, vp, C.c_int, vp, u32, C.POINTER(C.c_uint64), vp, vp, vp, u32]
P.gpucsum_set_inner.argtypes = [vp]
R.refs_config(0x0100000A)
T = C.CDLL(os.path.join(ROOT, "tools", "libburst_timer.so"))
T.bt_run.argtypes = [vp, vp, vp, vp, u32, vp, vp, u32, vp]


def vtab(lib, name):
    return C.addressof(C.c_char.in_dll(lib, name))


BURST, L = 64, 1500
BURSTS = int(os.environ.get("RXP_BURSTS", "400"))
n = BURST * BURSTS
src, stride = synth.fixed_frames(n, L, seed=0x5A)
off = np.arange(n, dtype=np.uint64) * stride
lens = np.full(n, L, dtype=np.uint16)
Oracle().compute_batch(src, off, lens)
bad = synth.corrupt(src, off, lens, frac_log2=6, seed=0x5B)
room = np.zeros(src.nbytes + 8192, np.uint8)           # page-aligned (registrable) copy
base = (-room.ctypes.data) % 4096
frames = room[base:base + src.nbytes]


def run(iom, ctx, registered):
    frames[:] = src                                    # fresh frames (the side effect writes)
    H.synth_reset(BURST)
    assert H.synth_set_rx(frames.ctypes.data, off.ctypes.data, lens.ctypes.data, n) == 0
    rx_bytes = C.c_uint64()
    rx_base = H.synth_rx_base(C.byref(rx_bytes))       # the NIC's RX rooms (its "mbuf pool")
    if registered:
        gpucsum.check(P.gcs_host_register(vp(rx_base), rx_bytes.value), "register")
    blocked = np.zeros(BURSTS, np.float64)
    burst = np.zeros(BURSTS, np.float64)
    recv = np.zeros(BURSTS, np.float64)
    disp = np.zeros(n, np.uint8)
    errs = C.c_uint64()
    try:
        assert R.refs_rx_loop_timed(iom, ctx, 0, disp.ctypes.data, n, C.byref(errs),
                                    blocked.ctypes.data, burst.ctypes.data, recv.ctypes.data,
                                    BURSTS) == n
    finally:
        if registered:
            gpucsum.check(P.gcs_host_unregister(vp(rx_base)), "unregister")
    b, w, rv = blocked[20:], burst[20:], recv[20:]     # past the first bursts' warm-up
    return {"blocked_us_median": float(np.median(b)), "blocked_us_p90": float(np.percentile(b, 90)),
            "recv_pkts_us_median": float(np.median(rv)),
            "burst_us_median": float(np.median(w)), "rx_errors": int(errs.value)}


def direct(registered, same):
    """gcs_verify_ptrs on each burst's 64 frames through the burst server, no
    decorator and no RX loop (same: burst 0's frames every time, as bench
    plugin_bursts)."""
    frames[:] = src
    ctx = gpucsum.Context(0, max_frames=4096, max_bytes=8 << 20)
    ctx.set_burst_server(True)                         # as the plugin's contexts
    verdict = np.zeros(BURST, np.uint8)
    ln = np.full(BURST, L, np.uint16)
    t = np.zeros(BURSTS, np.float64)
    fn = C.cast(P.gcs_verify_ptrs, vp)
    if registered:
        gpucsum.check(P.gcs_host_register(vp(frames.ctypes.data), frames.nbytes), "register")
    try:
        for k in range(BURSTS):
            j = 0 if same else k
            ptrs = (vp * BURST)(*[frames.ctypes.data + int(off[j * BURST + i]) for i in range(BURST)])
            gpucsum.check(T.bt_run(fn, ctx.h, ptrs, ln.ctypes.data, BURST, verdict.ctypes.data,
                                   None, 1, t[k:].ctypes.data), "verify")
    finally:
        if registered:
            gpucsum.check(P.gcs_host_unregister(vp(frames.ctypes.data)), "unregister")
        ctx.close()
    return {"verify_us_median": float(np.median(t[20:])), "verify_us_p90": float(np.percentile(t[20:], 90))}


out = {"workload": f"{BURSTS} bursts of {BURST} x {L}B TCP frames ({len(bad)} corrupted) through "
                   "the reference's own RX code (core.c loop, ProcessPacket); medians over bursts "
                   "20..",
       "timer": "C clock_gettime around recv_pkts and each get_rptr (blocked) and around the "
                "whole burst",
       "blocked": "time the mTCP thread spends inside recv_pkts + get_rptr per burst"}
ctx = C.create_string_buffer(64)
out["software_path"] = run(vtab(H, "synth_module_func"), C.addressof(ctx), False)
# the same software path over REGISTERED rooms: the host memory the fastest
# GPU rows use (compare GPU and CPU bursts on matched rooms)
out["software_path_registered"] = run(vtab(H, "synth_module_func"), C.addressof(ctx), True)
MODES = [(False, g, "host") for g in ("0", "8", "16", "32", "64")] + \
        [(False, g, "device") for g in ("8", "16", "32")] + \
        [(True, g, "host") for g in ("0", "8", "16", "32")]
for registered, group, stage in MODES:
    os.environ["GPUCSUM_RX_GROUP"] = group
    os.environ["GPUCSUM_TX_GROUP"] = "0"
    os.environ["GCS_ASYNC_STAGE"] = stage
    assert P.gpucsum_set_inner(vtab(H, "synth_module_func")) == 0
    iom = vtab(P, "gpucsum_module_func")
    dctx = C.create_string_buffer(64)
    assert H.mini_start(iom, C.addressof(dctx)) == 0
    try:
        r = run(iom, C.addressof(dctx), registered)
    finally:
        H.mini_stop(iom, C.addressof(dctx))
    assert r["rx_errors"] == out["software_path"]["rx_errors"], (r, out["software_path"])
    out[f"{'registered' if registered else 'pageable'}_group{group}"
        + ("_devstage" if stage == "device" else "")] = r
for registered in (False, True):
    for same in (False, True):
        out[f"direct_{'registered' if registered else 'pageable'}{'_same' if same else ''}"] = \
            direct(registered, same)
print(json.dumps(out))
