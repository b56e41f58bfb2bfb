"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 host path used by bench.py:
batch sharding, the pooled-embedding all-gather and the max-over-ranks timing."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from videoprism import distributed


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    r, lr, w = distributed.init("gloo")
    assert (r, lr, w) == (rank, rank, world)
    lo, hi = distributed.shard_range(64, r, w)
    local = torch.arange(lo, hi, dtype=torch.float32)[:, None].repeat(1, 3)
    gathered = distributed.all_gather_rows(local, w)
    t = distributed.max_over_ranks(float(rank + 1))
    distributed.barrier()
    q.put((rank, lo, hi, gathered[:, 0].tolist(), t))
    dist.destroy_process_group()


def test_shard_range_partitions():
    for B in (1, 7, 32, 256):
        for W in (1, 2, 3, 8):
            spans = [distributed.shard_range(B, r, W) for r in range(W)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(spans[i][1] == spans[i + 1][0] for i in range(W - 1))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.timeout(120)
def test_gloo_world2_gather_and_timing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, lo, hi, rows, t in res:
        assert rows == [float(i) for i in range(64)]   # every rank sees all clips in order
        assert t == 2.0                                  # max over ranks
    assert [(lo, hi) for _, lo, hi, _, _ in res] == [(0, 32), (32, 64)]
