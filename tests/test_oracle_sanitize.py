"""The oracle under AddressSanitizer + UBSan (the reference has
no sanitizer runs and its folds read past short buffers, tcp_in.c:1231).

oracle/sanitize_check.c fuzzes every per-frame and batch entry point of
oracle/csum_ref.h with seeded, mutated mTCP frames, each in its own
exactly-sized heap block, so any access outside a frame aborts the run.
CPU only; test infrastructure checking test infrastructure.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def fuzzer():
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True)
    return os.path.join(ROOT, "oracle", "_san", "sanitize_check")


@pytest.mark.parametrize("seed", [1, 0x6d746370, 0xBAD5EED])
def test_oracle_is_memory_safe_on_malformed_frames(fuzzer, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([fuzzer, "6000", str(seed)], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "sanitize_check ok" in r.stdout
    assert "runtime error" not in r.stderr
