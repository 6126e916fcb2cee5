"""Per-GPU sharding of frame batches.

Frames are independent, so N GPUs take N contiguous frame ranges with no
data-path collective -- the GPU analogue of mTCP's per-core RSS shards
(core.c:1153-1245, dpdk_module.c:716-746).  The only torch.distributed calls
on the bench path are a barrier and a max-reduction of the elapsed time.
"""
from __future__ import annotations

import os


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) frame range of `rank`; sizes differ by at most 1."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    return n_total * rank // world, n_total * (rank + 1) // world


def device_for_thread(ordinal: int, n_gpus: int) -> int:
    """mTCP thread k -> GPU k mod n (gpucsum_module.c init_handle)."""
    return ordinal % n_gpus


def env_world() -> tuple[int, int, int]:
    """(world, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def barrier(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(world: int, x: float, device: str = "cuda") -> float:
    """Slowest rank's value (the bench reports whole-job time = max)."""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_per_rank(world: int, values: list[float], device: str = "cuda") -> list[list[float]]:
    """Every rank's `values` (same length on all ranks), on every rank: the
    per-GPU report of the bench line (mTCP prints per-thread NETSTAT the same
    way, core.c:189-218).  Called outside the timed region."""
    if world == 1:
        return [list(values)]
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [p.cpu().tolist() for p in parts]


def aggregate_rate(frames_per_rank: int, world: int, steps: int, seconds: float) -> float:
    """Whole-job frames per second: all ranks' frames over the max-over-ranks time."""
    return frames_per_rank * world * steps / seconds
