"""Multi-GPU plumbing: one process per GPU, clips sharded by batch (weak scaling), and the
all-gather of pooled clip embeddings for the video-text step (BASELINE.json configs 4/5:
`similarities = video_emb @ text_emb.T`, reference README.md:81).  The encoder itself has no
cross-clip exchange (encoders.py:411-580), so the gather is the only collective.

On GPUs the gather runs through the library's own C-ABI collective, `vp_allgather` (RCCL over
xGMI, include/videoprism_hip.h): `Communicator` bootstraps a `vp_comm` per process from a unique
id that rank 0 creates and torch.distributed's store hands to every rank.  torch.distributed
itself is only the launcher's rendezvous plus the bench's barrier / max-over-ranks timing; with
the 'gloo' backend (CPU tests) the gather falls back to torch.distributed on CPU tensors.
"""

from __future__ import annotations

import ctypes
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
        if "MASTER_PORT" not in os.environ:
            raise RuntimeError("WORLD_SIZE > 1 needs MASTER_PORT (torch.distributed.run sets it; "
                               "bench.py --gpus N spawns its ranks with one)")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, local_rank, world


def shard_range(global_batch: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous clip range [lo, hi) of `rank`; sizes differ by at most one."""
    base, rem = divmod(global_batch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


class Communicator:
    """An RCCL communicator of the library (`vp_comm_*`), one per process, over all ranks of the
    initialised torch.distributed group."""

    def __init__(self, device: int):
        import torch.distributed as dist

        from . import _native
        lib = _native.load()
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.device = device
        n = lib.vp_comm_id_bytes()
        obj = [None]
        if self.rank == 0:
            buf = (ctypes.c_uint8 * n)()
            _native.call("vp_comm_unique_id", buf, n)
            obj = [bytes(buf)]
        dist.broadcast_object_list(obj, src=0)
        uid = (ctypes.c_uint8 * n).from_buffer_copy(obj[0])
        h = ctypes.c_void_p()
        _native.call("vp_comm_init", uid, n, self.world, self.rank, device, ctypes.byref(h))
        self._h = h

    def all_gather_rows(self, local, stream=None):
        """[b, D] (contiguous, on this rank's GPU) -> [world*b, D], rank-major, on every rank."""
        import torch

        from . import _native
        local = local.contiguous()
        out = torch.empty((self.world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        s = stream if stream is not None else torch.cuda.current_stream(local.device)
        _native.call("vp_allgather", self._h, ctypes.c_void_p(local.data_ptr()),
                     ctypes.c_void_p(out.data_ptr()), local.numel(), _native._prec(local),
                     ctypes.c_void_p(s.cuda_stream))
        return out

    def close(self) -> None:
        from . import _native
        if getattr(self, "_h", None) is not None and _native._lib is not None:
            _native._lib.vp_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def all_gather_rows(local, world: int, comm: Communicator | None = None):
    """[b, D] per rank -> [world*b, D] on every rank (equal b on all ranks).  GPU tensors go
    through the library's RCCL gather when a Communicator is given; otherwise (CPU / gloo)
    torch.distributed's all_gather_into_tensor."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return local
    if comm is not None and local.is_cuda:
        return comm.all_gather_rows(local)
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
