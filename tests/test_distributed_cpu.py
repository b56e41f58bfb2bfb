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
    # uneven and empty shards (global batch 3 / 1 over 2 ranks): padded to the largest shard for
    # the collective, padding rows dropped, rank-major order kept
    uneven = {}
    for B in (3, 1):
        ulo, uhi = distributed.shard_range(B, r, w)
        u = torch.arange(ulo, uhi, dtype=torch.float32)[:, None].repeat(1, 5)
        uneven[B] = distributed.all_gather_rows(u, w)[:, 0].tolist()
    distributed.barrier()
    q.put((rank, lo, hi, gathered[:, 0].tolist(), t, uneven))
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
    for rank, lo, hi, rows, t, uneven in res:
        assert rows == [float(i) for i in range(64)]   # every rank sees all clips in order
        assert t == 2.0                                  # max over ranks
        assert uneven == {3: [0.0, 1.0, 2.0], 1: [0.0]}
    assert [(lo, hi) for _, lo, hi, _, _, _ in res] == [(0, 32), (32, 64)]


def _bench_env():
    return {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK",
                                                             "MASTER_ADDR", "MASTER_PORT")}


def _bench_standin(workload, batch, env_update=None):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = _bench_env()
    for k, v in (env_update or {}).items():
        if v is None:
            env.pop(k, None)
        else:
            env[k] = v
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--standin",
                        "--workload", workload, "--batch", str(batch), "--frames", "2", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=150, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    return lines[0]


@pytest.mark.timeout(200)
def test_bench_spawns_world2_base_gather():
    """`bench.py --gpus 2` without a launcher spawns 2 ranks and drives its real step logic (pool ->
    gather) with the CPU stand-in forward: rank-major rows of all 2*b clips, n_gpus == 2."""
    line = _bench_standin("base", 2, {"HSA_ENABLE_IPC_MODE_LEGACY": None})
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 4
    chk = line["standin_check"]
    assert chk["gathered_shape"] == [4, 768] and chk["row_order_ok"]
    # the parent had HSA_ENABLE_IPC_MODE_LEGACY unset: the spawned ranks get 0 (dmabuf IPC)
    assert chk["ipc_mode_legacy"] == "0"


def test_rank_env_keeps_an_explicit_ipc_mode():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    env = bench.rank_env(1, 4, 29500, base={"PATH": "/bin"})
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"]) == ("1", "1", "4")
    assert (env["MASTER_ADDR"], env["MASTER_PORT"]) == ("127.0.0.1", "29500")
    assert bench.rank_env(0, 2, 1, base={"HSA_ENABLE_IPC_MODE_LEGACY": "1"})["HSA_ENABLE_IPC_MODE_LEGACY"] == "1"


@pytest.mark.timeout(200)
def test_bench_spawns_world2_lvt_similarity():
    """LvT step: video embeddings -> gather -> similarity against the replicated text queries;
    the similarity covers every clip of both ranks ([2*b, Q], README.md:81)."""
    line = _bench_standin("lvt_base", 3)
    assert line["n_gpus"] == 2
    chk = line["standin_check"]
    assert chk["gathered_shape"] == [6, 768] and chk["row_order_ok"]
    assert chk["similarity_shape"] == [6, 8]


@pytest.mark.timeout(200)
def test_bench_spawn_stops_siblings_of_a_dead_rank():
    """A rank that dies before the rendezvous (here: rank 1 exits with 3 right after start-up)
    must not leave rank 0 blocked in init_process_group and the parent in wait(): the parent
    polls every child, stops the survivor and returns the failing code well inside the timeout."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--standin",
                        "--batch", "2", "--frames", "2", "--steps", "1", "--warmup", "0",
                        "--fail-rank", "1", "--spawn-timeout", "90"],
                       capture_output=True, text=True, timeout=150, env=_bench_env())
    dt = time.monotonic() - t0
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert dt < 60, dt
    assert "stopping the others" in r.stderr


@pytest.mark.timeout(200)
def test_bench_spawn_timeout():
    """The overall timeout ends a spawned run that does not finish (both ranks alive, rank 1
    never joins: it sleeps past the timeout) with code 124, both ranks stopped."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--standin",
                        "--batch", "2", "--frames", "2", "--steps", "1", "--warmup", "0",
                        "--hang-rank", "1", "--spawn-timeout", "8"],
                       capture_output=True, text=True, timeout=150, env=_bench_env())
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
