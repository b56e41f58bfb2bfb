"""Probe: can two ranks share one GPU in an RCCL communicator on this box?  (The multi-GPU all-gather has only
run on a 1-rank communicator; a 2-rank communicator on one device would exercise it on real hardware.)
Run: python tools/gpu/rccl_same_device_probe.py  -- spawns 2 ranks (gloo rendezvous on 127.0.0.1)."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port, env_extra):
    os.environ.update(env_extra)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda:0"))
        x = torch.full((4,), float(rank + 1), device="cuda:0")
        out = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(out, x)
        torch.cuda.synchronize()
        print(f"rank {rank}: all_gather ok {[float(o[0]) for o in out]}", flush=True)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: {type(e).__name__}: {str(e)[:300]}", flush=True)


if __name__ == "__main__":
    extra = dict(a.split("=", 1) for a in sys.argv[1:])
    mp.start_processes(worker, args=(2, 29531, extra), nprocs=2, start_method="spawn")
