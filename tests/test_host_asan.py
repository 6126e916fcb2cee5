"""Host code under sanitizers (GPU sanitizers are not available on this pool,
so only the host side is instrumented).  tests/plugin/asan_driver and
tsan_driver, built by __graft_entry__.build() from tests/plugin/Makefile.asan,
drive libmtcp_gpucsum's host entry points (staging slots, gather pool, burst
server, registered regions) and the io_module decorator, checking every result
against the oracle:
  asan_driver  AddressSanitizer + UBSan: any host memory error or undefined
               behaviour aborts the run
  tsan_driver  ThreadSanitizer over the threaded parts (one context per thread,
               the gather pool, the burst server's host side); races inside the
               uninstrumented ROCm runtime are suppressed (tests/plugin/tsan.supp)
"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
PLUGIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "plugin")


def run_driver(name, env_extra):
    path = os.path.join(PLUGIN, name)
    if not os.path.exists(path):
        pytest.fail(f"tests/plugin/{name} missing: run __graft_entry__.build() first")
    env = dict(os.environ, **env_extra)
    p = subprocess.run([path], cwd=PLUGIN, env=env, capture_output=True, text=True, timeout=240)
    out = p.stdout + p.stderr
    assert p.returncode == 0 and "HOST DRIVER OK" in p.stdout, out[-4000:]
    for part in ("part 1", "part 2", "part 3", "part 4", "part 5", "part 6"):
        assert part in p.stdout
    return out


def test_host_code_under_asan_ubsan():
    out = run_driver("asan_driver", {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
                                     "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]


def test_host_code_under_tsan():
    out = run_driver("tsan_driver", {"TSAN_OPTIONS": "halt_on_error=1:suppressions=tsan.supp"})
    assert "WARNING: ThreadSanitizer" not in out, out[-4000:]
