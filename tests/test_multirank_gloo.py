"""N>1 path on CPU: world_size-2 gloo processes shard a frame batch by
contiguous ranges (mtcp_amd.shard), each checks its shard (the oracle stands
in for the GPU kernel: no GPU here), and the gathered per-rank verdicts must
equal the whole-batch verdicts; the timing reduction is the max over ranks.
"""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, json
sys.path.insert(0, {root!r}); sys.path.insert(0, os.path.join({root!r}, "tests"))
import numpy as np, torch, torch.distributed as dist
from mtcp_amd import synth, shard
from oracle_lib import Oracle

dist.init_process_group("gloo")
world, rank, _ = shard.env_world()
n, L = 5003, 1500
buf, stride = synth.fixed_frames(n, L, seed=42)
O = Oracle()
O.compute_fixed(buf, stride, L, n)
bad = synth.corrupt(buf, np.arange(n, dtype=np.uint64) * stride, np.full(n, L), frac_log2=5, seed=1)
lo, hi = shard.shard_range(n, rank, world)
mine = O.verify_fixed(buf[lo * stride:hi * stride].copy(), stride, L, hi - lo)
sizes = [shard.shard_range(n, r, world) for r in range(world)]
m = max(h - l for l, h in sizes)          # gloo all_gather wants equal sizes: pad
parts = [torch.zeros(m, dtype=torch.uint8) for _ in sizes]
padded = torch.zeros(m, dtype=torch.uint8)
padded[: hi - lo] = torch.from_numpy(mine)
dist.all_gather(parts, padded)
whole = O.verify_fixed(buf, stride, L, n)
got = torch.cat([p[: h - l] for p, (l, h) in zip(parts, sizes)]).numpy()
ok = np.array_equal(got, whole)
t = shard.max_over_ranks(world, float(rank + 1), device="cpu")
per = shard.gather_per_rank(world, [float(rank), float(hi - lo), float((mine != 0).sum())],
                            device="cpu")
shard.barrier(world)
if rank == 0:
    print(json.dumps({{"ok": bool(ok), "t": t, "bad": int((whole != 0).sum()), "nbad": len(bad),
                      "per": per,
                      "rate": shard.aggregate_rate(hi - lo, world, 1, t)}}))
dist.destroy_process_group()
"""


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_partitions():
    from mtcp_amd import shard
    for n in (0, 1, 7, 1 << 20, 1 << 22):
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1
    assert [shard.device_for_thread(k, 8) for k in range(10)] == [0, 1, 2, 3, 4, 5, 6, 7, 0, 1]
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_two_rank_gloo_shards_equal_whole(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(script)]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    import json
    res = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["ok"]
    assert res["t"] == 2.0                       # max over ranks
    assert res["bad"] == res["nbad"] > 0
    per = res["per"]                             # per-rank report, gathered
    assert [p[0] for p in per] == [0.0, 1.0]
    assert sum(p[1] for p in per) == 5003 and sum(p[2] for p in per) == res["bad"]
