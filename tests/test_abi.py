"""The C-ABI boundary without a GPU: the library loads, exports every entry
point include/*.h declares, verdict/status numbering matches the oracle, and
argument validation fails loudly (no compute call is made)."""
import ctypes as C
import glob
import os
import re
import subprocess

import pytest

from mtcp_amd import gpucsum

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b((?:gcs|gpucsum)_\w+)\s*\(", src, re.M):
            names.add(m.group(1))
        for m in re.finditer(r"^extern\s+[\w ]+\s+((?:gcs|gpucsum)_\w+)\s*;", src, re.M):
            names.add(m.group(1))
    return sorted(names)


def exported_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert "gcs_verify_fixed_dev" in names and "gcs_tcp_checksum_dev" in names
    syms = exported_symbols(gpucsum.LIB_PATH)
    missing = [n for n in names if n not in syms]
    assert not missing, missing
    L = gpucsum.lib()
    for n in names:
        assert getattr(L, n) is not None


def test_abi_version_and_strerror():
    L = gpucsum.lib()
    assert L.gcs_abi_version() == gpucsum.K["GCS_ABI_VERSION"] == 2
    assert L.gcs_strerror(-1) == b"invalid argument"
    assert L.gcs_strerror(0) == b"ok"


def test_codes_match_oracle():
    src = open(os.path.join(ROOT, "oracle", "csum_ref.h")).read()
    ref = {m.group(1): int(m.group(2)) for m in re.finditer(r"REF_(V_\w+|TX_\w+)\s*=\s*(\d+)", src)}
    K = gpucsum.K
    for k, v in ref.items():
        assert K["GCS_" + k] == v, k
    assert K["GCS_VF_ZERO_BAD_TCP_CHECK"] == 1
    assert K["GCS_VF_ICMP"] == 2 and K["GCS_CF_ICMP"] == 2
    for k in ("V_ICMP_OK", "V_ICMP_BADCSUM", "TX_ICMP_OK", "TX_BAD_ICMPLEN"):
        assert k in ref


def test_error_predicate_excludes_icmp_verdicts():
    """ICMP checksum failures are not mTCP errors (ProcessICMPPacket returns
    TRUE, icmp.c:140): the plugin must not drop them."""
    src = open(os.path.join(ROOT, "include", "mtcp_gpucsum.h")).read()
    m = re.search(r"#define GCS_V_IS_ERROR\(v\)\s*(.+)", src)
    pred = eval("lambda v: " + m.group(1).replace("&&", " and ").replace("||", " or "))
    K = gpucsum.K
    errs = {K[k] for k in K if k.startswith("GCS_V_") and k != "GCS_V_IS_ERROR" and
            pred(K[k])}
    assert errs == {2, 3, 6, 7, 8, 9}


def test_argument_validation_without_gpu():
    L = gpucsum.lib()
    # NULL context / bad stride are rejected before any HIP call
    assert L.gcs_verify_fixed_dev(None, None, 64, 64, 1, None, 0, None) == gpucsum.K["GCS_EINVAL"]
    assert L.gcs_ctx_destroy(None) == gpucsum.K["GCS_EINVAL"]
    p = C.c_void_p()
    assert L.gcs_ctx_create(None, 0, 0, 0) == gpucsum.K["GCS_EINVAL"]
    assert L.gcs_device_count(None) == gpucsum.K["GCS_EINVAL"]
    assert L.gcs_ctx_set_rss(None, None, 0, 4, 0) == gpucsum.K["GCS_EINVAL"]
    assert L.gcs_classify_fixed_dev(None, None, 64, 64, 1, None, None, None, 0, None) == \
        gpucsum.K["GCS_EINVAL"]
    assert L.gcs_rss_dev(None, None, None, None, None, 1, None, None, None) == \
        gpucsum.K["GCS_EINVAL"]


def test_no_device_here_is_reported_not_faked():
    """Without a GPU, creating a context fails with an error code: there is
    no CPU fallback behind the ABI."""
    if gpucsum.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(gpucsum.GcsError):
        gpucsum.Context(0)


def test_product_does_not_link_oracle():
    out = subprocess.run(["ldd", gpucsum.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out and "ref_mtcp" not in out
    syms = exported_symbols(gpucsum.LIB_PATH)
    assert not any(s.startswith(("ref_", "refx_", "TCPCalcChecksum")) for s in syms)


@pytest.mark.parametrize("defrag", [False, True], ids=["dpdk", "dpdk_IP_DEFRAG"])
def test_set_inner_picks_caps_for_mtcp_modules(tmp_path, defrag):
    """gpucsum_set_inner recognises mTCP's own modules through weak references:
    netmap's get_wptr transmits (TX_EAGER, netmap_module.c:149-160); DPDK frames
    over one MTU frame are ENABLELRO chains (RX_CHAINED, dpdk_module.c:44-48,
    112-135); a DPDK module built with IP_DEFRAG (the integration patch defines
    dpdk_module_ip_defrag there) feeds its reassembly table on every get_rptr
    call (dpdk_module.c:474-529), so it gets RX_ONCE.  The modules are defined
    in an -rdynamic executable, as a linked mTCP exports them; no GPU call is
    made."""
    exe = str(tmp_path / "inner_caps")
    subprocess.run(["gcc", "-O1", "-rdynamic", "-I", os.path.join(ROOT, "include")] +
                   (["-DWITH_IP_DEFRAG"] if defrag else []) +
                   [os.path.join(ROOT, "tests", "plugin", "inner_caps.c"),
                    "-L", os.path.dirname(gpucsum.LIB_PATH), "-lmtcp_gpucsum",
                    "-Wl,-rpath," + os.path.dirname(gpucsum.LIB_PATH), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    got = dict(zip(out[0::2], map(int, out[1::2])))
    assert got == {"dpdk": 4 if defrag else 2, "netmap": 1, "other": 0, "set": 2}


def test_host_register_rejects_bad_regions():
    """Regions of 64 GiB or more cannot be described to the burst server
    (ServerReqB.bytes16 is a u32) and are refused before any HIP call."""
    L = gpucsum.lib()
    buf = C.create_string_buffer(64)
    EINVAL = gpucsum.K["GCS_EINVAL"]
    assert L.gcs_host_register(None, 64) == EINVAL
    assert L.gcs_host_register(buf, 0) == EINVAL
    assert L.gcs_host_register(buf, 64 << 30) == EINVAL
