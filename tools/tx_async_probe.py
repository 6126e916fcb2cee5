"""How long send_pkts blocks the mTCP thread per TX burst, with and without the
plugin's fill-as-you-go (GPUCSUM_TX_GROUP), through the mTCP-shaped TX loop
(tests/plugin/mini_mtcp.c mini_tx_timed: get_wptr, headers + payload memcpy,
PKT_TX_TCPIP_CSUM, send_pkts every 64 frames, core.c:846-848) over the
synthetic NIC module, whose TX rooms are pageable or registered (in place).
The software path (the module alone, mTCP folding on the CPU) is timed the
same way, over pageable and over registered rooms (software_path_registered:
the same host memory as the registered GPU rows).  Prints one JSON object (tools/, not product)."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process: torch first)
from mtcp_amd import gpucsum, synth  # noqa: E402

vp = C.c_void_p
P = gpucsum.lib()
H = C.CDLL(os.path.join(ROOT, "tests", "plugin", "libplugin_harness.so"))
H.synth_reset.argtypes = [C.c_uint32]
H.synth_tx_base.argtypes = [C.POINTER(C.c_uint64)]
H.synth_tx_base.restype = vp
H.synth_tx_sent.restype = C.c_uint32
H.mini_start.argtypes = [vp, vp]
H.mini_stop.argtypes = [vp, vp]
H.mini_tx_timed.argtypes = [vp, vp, C.c_int, vp, vp, vp, C.c_uint32, C.c_uint32, vp, vp]
P.gpucsum_set_inner.argtypes = [vp]


def vtab(lib, name):
    return C.addressof(C.c_char.in_dll(lib, name))


BURST, L = 64, 1500
BURSTS = int(os.environ.get("TXP_BURSTS", "400"))
n = BURST * BURSTS
frames, stride = synth.fixed_frames(n, L, seed=0x7A)
off = np.arange(n, dtype=np.uint64) * stride
lens = np.full(n, L, dtype=np.uint16)


def run(iom, ctx, registered):
    H.synth_reset(BURST)
    base = None
    if registered:
        nb = C.c_uint64()
        base = H.synth_tx_base(C.byref(nb))
        gpucsum.check(P.gcs_host_register(vp(base), nb.value), "register")
    send = np.zeros(BURSTS, np.float64)
    burst = np.zeros(BURSTS, np.float64)
    try:
        assert H.mini_tx_timed(iom, ctx, 0, frames.ctypes.data, off.ctypes.data, lens.ctypes.data,
                               n, BURST, send.ctypes.data, burst.ctypes.data) == n
        assert H.synth_tx_sent() == n
    finally:
        if base:
            gpucsum.check(P.gcs_host_unregister(vp(base)), "unregister")
    s, b = send[20:], burst[20:]                  # past the first bursts' warm-up
    return {"send_pkts_us_median": float(np.median(s)), "send_pkts_us_p90": float(np.percentile(s, 90)),
            "burst_us_median": float(np.median(b))}


out = {"workload": f"{BURSTS} bursts of {BURST} x {L}B TCP frames through mini_tx_timed "
                   "(headers + payload memcpy per frame, PKT_TX_TCPIP_CSUM, send_pkts per burst); "
                   "medians over bursts 20..",
       "timer": "C clock_gettime around each send_pkts and each burst"}
ctx = C.create_string_buffer(64)
out["software_path"] = run(vtab(H, "synth_module_func"), C.addressof(ctx), False)
# the same software path over REGISTERED rooms: the host memory the fastest
# GPU rows use (compare GPU and CPU bursts on matched rooms)
out["software_path_registered"] = run(vtab(H, "synth_module_func"), C.addressof(ctx), True)
MODES = [(False, g, "host") for g in ("0", "8", "16")] + [(False, "8", "device"), (False, "16", "device")] + \
        [(True, g, "host") for g in ("0", "8", "16")] + [(True, None, "host"), (False, None, "host")] + \
        [(True, "16", "regstage")]
if os.environ.get("TXP_SMALL_GROUPS"):
    MODES += [(False, g, st) for g in ("2", "4") for st in ("host", "device")]
for registered, group, stage in MODES:
        if group is None:                          # the plugin's default
            os.environ.pop("GPUCSUM_TX_GROUP", None)
        else:
            os.environ["GPUCSUM_TX_GROUP"] = group
        os.environ["GCS_ASYNC_STAGE"] = "device" if stage == "regstage" else stage
        os.environ["GCS_ASYNC_REGISTERED"] = "stage" if stage == "regstage" else "inplace"
        assert P.gpucsum_set_inner(vtab(H, "synth_module_func")) == 0
        iom = vtab(P, "gpucsum_module_func")
        dctx = C.create_string_buffer(64)
        assert H.mini_start(iom, C.addressof(dctx)) == 0
        try:
            r = run(iom, C.addressof(dctx), registered)
        finally:
            H.mini_stop(iom, C.addressof(dctx))
        out[f"{'registered' if registered else 'pageable'}_group{group or 'default'}"
            + {"device": "_devstage", "regstage": "_devstage"}.get(stage, "")] = r
print(json.dumps(out))
