"""Multi-GPU plumbing: one process per GPU, clips sharded by batch (weak scaling), and the
all-gather of pooled clip embeddings for the video-text step (BASELINE.json configs 4/5:
`similarities = video_emb @ text_emb.T`, reference README.md:81).  The encoder itself has no
cross-clip exchange (encoders.py:411-580), so the gather is the only collective.

On GPUs the gather runs through the library's own C-ABI collective, `vp_allgather` (RCCL over
xGMI, include/videoprism_hip.h): `Communicator` bootstraps a `vp_comm` per process from a unique
id that rank 0 creates and torch.distributed's store hands to every rank.  torch.distributed
itself is a CPU (`gloo`) group: the launcher's rendezvous, the id broadcast, the row-count
exchange of uneven shards and the bench's barrier / max-over-ranks timing -- so the library's
`vp_comm` is each rank's only RCCL communicator.  With CPU tensors (tests) the gather falls
back to torch.distributed's all_gather over gloo.
"""

from __future__ import annotations

import ctypes
import os
import warnings


def env_world() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def local_device(local_rank: int) -> int:
    """The HIP device index of this rank: LOCAL_RANK when the process sees every GPU of the node
    (torch.distributed.run's default), 0 when a launcher narrowed it to one GPU
    (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES per rank); anything else is a launch error."""
    import torch
    n = torch.cuda.device_count()
    if local_rank < n:
        return local_rank
    if n == 1:
        return 0
    raise RuntimeError(f"LOCAL_RANK {local_rank} but only {n} visible HIP devices")


def init(backend: str = "gloo", timeout_s: float = 600.0):
    """Join the launcher's process group (a CPU `gloo` group by default: GPU data moves only
    through the library's RCCL communicator).  A rank that never arrives fails the others after
    `timeout_s` instead of blocking them forever."""
    import datetime

    import torch.distributed as dist
    rank, local_rank, world = env_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            raise RuntimeError("WORLD_SIZE > 1 needs MASTER_PORT (torch.distributed.run sets it; "
                               "bench.py --gpus N spawns its ranks with one)")
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s))
    return rank, local_rank, world


def shard_range(global_batch: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous clip range [lo, hi) of `rank`; sizes differ by at most one (a rank may get
    none when global_batch < world)."""
    base, rem = divmod(global_batch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def _row_counts(n: int, world: int) -> list[int]:
    """Every rank's row count (host exchange over the CPU process group)."""
    import torch.distributed as dist
    counts = [None] * world
    dist.all_gather_object(counts, int(n))
    return [int(c) for c in counts]


class Communicator:
    """An RCCL communicator of the library (`vp_comm_*`), one per process, over all ranks of the
    initialised torch.distributed group.  Close it explicitly (`close()` or a `with` block)
    before the process group is destroyed: RCCL teardown synchronises with the peers, which
    garbage collection at interpreter exit cannot order."""

    def __init__(self, device: int):
        import torch.distributed as dist

        from . import _native
        lib = _native.load()
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.device = device
        self._h = None
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

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def all_gather_rows(self, local, stream=None, counts: list[int] | None = None):
        """[b_r, D] (on this rank's GPU) -> [sum_r b_r, D], rank-major, on every rank.

        RCCL's all-gather needs one count on every rank, so shards of different sizes (including
        empty ones: `shard_range` when the global batch does not divide by the world) are padded
        to the largest shard, gathered, and the padding rows dropped.  `counts` (every rank's
        b_r) skips the host exchange when the caller already knows them; a `counts` entry that
        disagrees with this rank's rows raises before any collective is entered."""
        import torch

        from . import _native
        if self._h is None:
            raise RuntimeError("communicator is closed")
        local = local.contiguous()
        b = int(local.shape[0])
        if counts is None:
            counts = _row_counts(b, self.world)
        if len(counts) != self.world or counts[self.rank] != b:
            raise ValueError(f"row counts {counts} do not match this rank's {b} rows")
        bmax = max(counts)
        tail = tuple(local.shape[1:])
        if bmax == 0:
            return torch.empty((0,) + tail, dtype=local.dtype, device=local.device)
        # Stream order: `local` was produced on the caller's current stream; the padding copy, the
        # gather and the unpadding all run on `s`, which first waits for the current stream; the
        # current stream then waits for `s`, so the caller can use the result right away.  Tensors
        # allocated on one stream and used on the other are recorded on it, so the caching
        # allocator does not hand their memory out while the other stream may still use it.
        cur = torch.cuda.current_stream(local.device)
        s = stream if stream is not None else cur
        side = s != cur
        if side:
            s.wait_stream(cur)
            local.record_stream(s)
        with torch.cuda.stream(s):
            send = local
            if b != bmax:
                send = torch.zeros((bmax,) + tail, dtype=local.dtype, device=local.device)
                send[:b].copy_(local)
            full = torch.empty((self.world * bmax,) + tail, dtype=local.dtype, device=local.device)
            _native.call("vp_allgather", self._h, ctypes.c_void_p(send.data_ptr()),
                         ctypes.c_void_p(full.data_ptr()), send.numel(), _native._prec(local),
                         ctypes.c_void_p(s.cuda_stream))
            if all(c == bmax for c in counts):
                out = full
            else:
                out = torch.cat([full[r * bmax:r * bmax + c] for r, c in enumerate(counts)])
        if side:
            cur.wait_stream(s)
            out.record_stream(cur)
        return out

    def close(self) -> None:
        from . import _native
        if getattr(self, "_h", None) is not None and _native._lib is not None:
            _native._lib.vp_comm_destroy(self._h)
        self._h = None

    def __del__(self):
        # no collective teardown from the garbage collector (it may run after the peers exited)
        if getattr(self, "_h", None) is not None:
            warnings.warn("videoprism.distributed.Communicator was not closed; its RCCL "
                          "communicator is leaked", ResourceWarning, stacklevel=1)


def all_gather_rows(local, world: int, comm: Communicator | None = None,
                    counts: list[int] | None = None):
    """[b_r, D] per rank -> [sum_r b_r, D] rank-major on every rank; shards may differ in size
    (see Communicator.all_gather_rows).  GPU tensors go through the library's RCCL gather when a
    Communicator is given; CPU tensors through torch.distributed's all_gather (gloo)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return local
    if comm is not None and local.is_cuda:
        return comm.all_gather_rows(local, counts=counts)
    local = local.contiguous()
    if counts is None:
        counts = _row_counts(int(local.shape[0]), world)
    bmax = max(counts)
    tail = tuple(local.shape[1:])
    send = local
    if local.shape[0] != bmax:
        send = torch.zeros((bmax,) + tail, dtype=local.dtype, device=local.device)
        send[:local.shape[0]].copy_(local)
    parts = [torch.empty_like(send) for _ in range(world)]
    dist.all_gather(parts, send)
    return torch.cat([p[:c] for p, c in zip(parts, counts)])


def max_over_ranks(value: float, device=None) -> float:
    """Max of a host float over all ranks (the CPU process group; `device` is ignored unless
    the group is an nccl one)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    dev = device if dist.get_backend() == "nccl" else None
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None) -> None:
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if device is not None and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()
