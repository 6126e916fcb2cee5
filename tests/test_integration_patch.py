"""INTEGRATION.md's mTCP patch, applied and built (no GPU).

integration/mtcp_gpucsum.patch is the change a maintainer applies to mTCP to
drop the decorator in: the `gpucsum` field in struct mtcp_config (mtcp.h), its
mtcp.conf key (config.c:635-640), the decorator wrapped around the configured
module in mtcp_init and MTCPRunThread (core.c:1187, :1639), the ENABLELRO
gather's module check (tcp_ring_buffer.c:15-21) and the build lines.

Here it is applied to a copy of the reference tree and every source of
libmtcp (mtcp/src/Makefile.in SRCS) is compiled with the reference flags
(Makefile.in:44-56) WITHOUT -DDISABLE_HWCSUM, with and without -DENABLELRO,
then linked with -Wl,--no-undefined against libmtcp_gpucsum.so: every symbol
the patched mTCP needs from the decorator resolves.  The NIC backends are
configured out (-DDISABLE_DPDK/PSIO/NETMAP: their SDKs are not in this image).
The reference tree is only read; nothing of it is kept.
"""
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

from mtcp_amd import gpucsum

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PATCH = os.path.join(ROOT, "integration", "mtcp_gpucsum.patch")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "mtcp", "src")),
                                reason="needs the reference tree (this container only)")

# mtcp/src/Makefile.in:44-56 (minus -Werror: see test_patch_adds_no_warnings)
REF_FLAGS = ["-m64", "-Wall", "-fPIC", "-fgnu89-inline", "-DNDEBUG", "-g", "-O3", "-DNETSTAT",
             "-DINFO", "-DDBGERR", "-DDBGCERR", "-D__USRLIB__", "-fcommon",
             "-DDISABLE_DPDK", "-DDISABLE_PSIO", "-DDISABLE_NETMAP"]
PATCHED = ("core.c", "config.c", "tcp_ring_buffer.c")


def copy_tree(dst):
    shutil.copytree(os.path.join(REF, "mtcp", "src"), os.path.join(dst, "mtcp", "src"))
    shutil.copytree(os.path.join(REF, "io_engine", "include"),
                    os.path.join(dst, "io_engine", "include"))
    os.makedirs(os.path.join(dst, "apps", "example"))
    shutil.copy(os.path.join(REF, "apps", "example", "Makefile.in"),
                os.path.join(dst, "apps", "example"))


def srcs(tree):
    mk = open(os.path.join(tree, "mtcp", "src", "Makefile.in")).read()
    m = re.search(r"^SRCS = (.*?)\n\n", mk, re.S | re.M)
    return m.group(1).replace("\\", " ").split()


def compile_one(tree, f, extra):
    src = os.path.join(tree, "mtcp", "src")
    obj = os.path.join(src, f[:-2] + ".o")
    r = subprocess.run(["gcc", *REF_FLAGS, *extra, "-I", os.path.join(src, "include"),
                        "-I", os.path.join(tree, "io_engine", "include"),
                        "-I", os.path.join(ROOT, "include"), "-c", os.path.join(src, f),
                        "-o", obj], capture_output=True, text=True)
    return f, r.returncode, r.stderr, obj


def warnings_of(stderr):
    # line numbers move with the patch: compare messages
    return {re.sub(r"^.*/([^/]+):\d+:\d+:", r"\1:", l).strip() for l in stderr.splitlines()
            if "warning:" in l}


@pytest.fixture(scope="module")
def trees(tmp_path_factory):
    base = tmp_path_factory.mktemp("mtcp")
    orig, patched = str(base / "orig"), str(base / "patched")
    copy_tree(orig)
    copy_tree(patched)
    r = subprocess.run(["patch", "-p1", "--forward", "--batch", "-i", PATCH], cwd=patched,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAILED" not in r.stdout and "offset" not in r.stdout.lower(), r.stdout
    return orig, patched


def test_patch_applies_cleanly(trees):
    _, patched = trees
    src = open(os.path.join(patched, "mtcp", "src", "core.c")).read()
    assert "gpucsum_module_func.load_module()" in src and "&gpucsum_module_func" in src
    assert "int gpucsum;" in open(os.path.join(patched, "mtcp", "src", "include", "mtcp.h")).read()


@pytest.mark.parametrize("lro", [False, True], ids=["plain", "ENABLELRO"])
def test_patched_libmtcp_builds_and_links(trees, lro):
    _, patched = trees
    extra = ["-DENABLELRO"] if lro else []
    with ThreadPoolExecutor(8) as ex:
        res = list(ex.map(lambda f: compile_one(patched, f, extra), srcs(patched)))
    failed = [(f, err) for f, rc, err, _ in res if rc]
    assert not failed, failed[:3]
    so = os.path.join(patched, "libmtcp_patched.so")
    libdir = os.path.dirname(gpucsum.LIB_PATH)
    r = subprocess.run(["gcc", "-shared", "-o", so, *[o for *_, o in res],
                        "-Wl,--no-undefined", "-L", libdir, "-lmtcp_gpucsum", "-lnuma",
                        "-lpthread", "-lrt"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    undef = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True,
                           text=True, check=True).stdout
    for sym in ("gpucsum_set_inner", "gpucsum_get_inner", "gpucsum_module_func"):
        assert sym in undef, sym                   # resolved from libmtcp_gpucsum.so
    if lro:
        assert "gpucsum_set_inner_caps" in undef


@pytest.mark.parametrize("lro", [False, True], ids=["plain", "ENABLELRO"])
def test_patch_adds_no_warnings(trees, lro):
    """The reference builds with -Werror.  Under this compiler (gcc 11) and
    the backends configured out, config.c already warns unpatched; the patch
    adds no warning to any file it touches, and core.c / tcp_ring_buffer.c,
    clean before, stay clean."""
    orig, patched = trees
    extra = ["-DENABLELRO"] if lro else []
    for f in PATCHED:
        _, rc0, e0, _ = compile_one(orig, f, extra)
        _, rc1, e1, _ = compile_one(patched, f, extra)
        assert rc0 == 0 and rc1 == 0, e1
        assert warnings_of(e1) <= warnings_of(e0), (f, warnings_of(e1) - warnings_of(e0))
    for f in ("core.c", "tcp_ring_buffer.c"):
        _, rc, err, _ = compile_one(patched, f, extra + ["-Werror"])
        assert rc == 0, err
