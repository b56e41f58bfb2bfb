"""Multi-GPU plumbing: one process per GPU, clips sharded by batch (weak scaling), and
the optional all-gather of pooled clip embeddings over RCCL for the video-text step
(BASELINE.json configs 4/5).  The encoder itself has no cross-clip exchange
(encoders.py:411-580), so the gather is the only collective.  torch.distributed with
backend 'nccl' is RCCL on ROCm; 'gloo' is used by the CPU tests.
"""

from __future__ import annotations

import os


def env_world() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def init(backend: str = "nccl"):
    import torch.distributed as dist
    rank, local_rank, world = env_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, local_rank, world


def shard_range(global_batch: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous clip range [lo, hi) of `rank`; sizes differ by at most one."""
    base, rem = divmod(global_batch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def all_gather_rows(local, world: int):
    """[b, D] per rank -> [world*b, D] on every rank (equal b on all ranks)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return local
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous())
    return out


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None) -> None:
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if device is not None and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()
