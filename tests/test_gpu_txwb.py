"""The TX fill's write-back modes (gcs_kernels.hip tx_wb, k_fixed_tx2 and
k_fixed_step): whole lines for the first GCS_TX_LINE_WB_MB of lines, then
non-temporal (default) or sc1 sector stores, or sectors throughout
(GCS_TX_HYBRID=off) -- every mode must fill exactly what the reference's
ip_out.c:143-173 / tcp_out.c:323-333 fill, through gcs_compute_fixed_dev and
through the fused gcs_step_fixed_dev.  The knobs are read once per process,
so each mode runs in a child process (one GPU process at a time), with a
1 MB line budget: frames [0, 8192) take lines, the rest sectors."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys
import numpy as np
import torch
sys.path.insert(0, "tests")
from mtcp_amd import gpucsum, synth
from oracle_lib import Oracle
O = Oracle()
n, L = 20000, 1500
tx, stride = synth.fixed_frames(n, L, seed=7)
rx, _ = synth.fixed_frames(n, L, seed=8)
off = np.arange(n, dtype=np.uint64) * stride
lens = np.full(n, L, dtype=np.uint16)
O.compute_batch(rx, off, lens)
bad = synth.corrupt(rx, off, lens, frac_log2=4, seed=9)
ref = tx.copy()
rst, rcs = O.compute_fixed(ref, stride, L, n)
rv = O.verify_batch(rx.copy(), off, lens)
out = {}
with gpucsum.Context(0) as c:
    d = torch.from_numpy(tx).cuda()
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cs = torch.zeros(n, dtype=torch.int32, device="cuda")
    c.compute_fixed(d, stride, L, n, st, cs)
    c.sync()
    out["fill"] = bool(np.array_equal(d.cpu().numpy(), ref) and
                       np.array_equal(st.cpu().numpy(), rst) and
                       np.array_equal(cs.cpu().numpy().view(np.uint32), rcs))
    d = torch.from_numpy(tx).cuda()
    r = torch.from_numpy(rx).cuda()
    v = torch.zeros(n, dtype=torch.uint8, device="cuda")
    c.step_fixed(d, stride, L, n, r, stride, L, n, v, st, cs)
    c.sync()
    out["step"] = bool(np.array_equal(d.cpu().numpy(), ref) and
                       np.array_equal(st.cpu().numpy(), rst) and
                       np.array_equal(v.cpu().numpy(), rv) and bool((rv[bad] != 0).all()))
    gpucsum.device_check(0)
print(json.dumps(out))
'''


@pytest.mark.parametrize("hybrid", ["nt", "sc1", "off"])
def test_fill_write_back_modes(hybrid):
    env = dict(os.environ, GCS_TX_LINE_WB_MB="1", GCS_TX_HYBRID=hybrid)
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"fill": True, "step": True}
