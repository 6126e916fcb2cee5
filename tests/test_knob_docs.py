"""Every environment knob the library and the plugin read is documented in
INTEGRATION.md (no GPU): a knob that only the source knows about is one a
deployment cannot find."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ["gcs_api.cpp", "gcs_kernels.hip", "gpucsum_module.c", "gcs_internal.h", "gcs_device.h"]


def knobs():
    found = set()
    for name in SOURCES:
        text = open(os.path.join(ROOT, "mtcp_amd", "csrc", name)).read()
        found |= set(re.findall(r'getenv\("([A-Z0-9_]+)"\)', text))
    return found


def test_every_knob_is_documented():
    found = knobs()
    assert len(found) >= 30, sorted(found)     # the scan itself works
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    missing = sorted(k for k in found if f"`{k}`" not in doc and f"{k}`" not in doc)
    assert not missing, missing
