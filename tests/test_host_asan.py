"""Host code under AddressSanitizer + UBSan (GPU sanitizers are not available on this
pool, so only the host side is instrumented): tests/plugin/asan_driver, built
by __graft_entry__.build() from tests/plugin/Makefile.asan, drives
libmtcp_gpucsum's host entry points (staging slots, gather pool, burst server,
registered regions) and the io_module decorator, checking every result against
the oracle.  ASan aborts the run on any host memory error, UBSan on undefined
behaviour."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(HERE, "plugin", "asan_driver")


def test_host_code_under_asan():
    if not os.path.exists(DRIVER):
        pytest.fail("tests/plugin/asan_driver missing: run __graft_entry__.build() first")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([DRIVER], cwd=os.path.dirname(DRIVER), env=env, capture_output=True,
                       text=True, timeout=240)
    out = p.stdout + p.stderr
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert p.returncode == 0 and "ASAN DRIVER OK" in p.stdout, out[-4000:]
    for part in ("part 1", "part 2", "part 3", "part 4", "part 5"):
        assert part in p.stdout
