#!/usr/bin/env python3
"""VideoPrism-Base bf16 forward throughput on MI355X (BASELINE.json metric/configs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload base|large|lvt_large|lvt_base] [--dtype bf16|f32]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one forward of the `videoprism_public_v1_base` FactorizedEncoder (bf16, random-init
weights of the real architecture) over B=32 synthetic clips [32,16,288,288,3] uniform[0,1)
already resident in HBM (configs[1]); for N>1 every rank runs its own 32 clips (weak scaling,
configs[3]: B=32*N) and the step includes the all-gather of the pooled, L2-normalised clip
embeddings through the library's RCCL collective (vp_allgather).  value = clips processed by all
ranks / max-over-ranks time.  Without torch.distributed.run, `--gpus N > 1` spawns the N ranks
itself (before any GPU call in the parent).

Also reported (one JSON line on rank 0):
  roofline     the dominant kernel's algorithmic FLOP (or byte) rate, from HIP events recorded
               on its launch stream inside the timed region, against the MI355X dense peak; its
               HBM `traffic` from a PMC record of the same kernel symbol and the same sources
               (the newest profiles/traffic_r*_<workload>.json whose source fingerprint matches,
               tools/pmc_traffic.sh), else null
  cpu_baseline the NumPy oracle (oracle/, fp32) on one clip on this host's cores (rank 0, N=1)

`--dtype f32` measures the same step in fprop_dtype=float32 (the reference's default, `get_model(name)`), against
the fp32 MFMA peak; the headline line is bf16.

`--standin` replaces the GPU forward by a small CPU function (gloo backend) so the multi-process
plumbing -- spawning, sharding, the gather's row order, the similarity shape, n_gpus -- can be
exercised on a machine without GPUs (tests/test_distributed_cpu.py).  It measures nothing.
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip parameters)
PEAK_F32_TFLOPS = 157.3     # MI355X fp32 MFMA (--dtype f32: the reference's default precision)
PEAK_HBM_GBS = 8000.0       # MI355X HBM3E spec (same table)
CPU_BASELINE_THREADS = 16   # the GPU box's CPU share per GPU


def gflop_per_clip(cfg: dict, T: int = 16, N: int = 256) -> float:
    """Algorithmic GFLOP per clip (2 flop/MAC): GEMMs + attention + patch embed."""
    D, F = cfg["model_dim"], cfg["mlp_dim"]
    Ls, Lt = cfg["num_spatial_layers"], cfg["num_temporal_layers"]
    P = cfg["patch_size"]
    tok = T * N
    gemm = (8 * D * D + 4 * D * F) * tok * (Ls + Lt)
    sp_att = 4 * N * N * D * T * Ls
    tp_att = 4 * T * T * D * N * Lt
    patch = 2 * P * P * 3 * D * tok
    return (gemm + sp_att + tp_att + patch) / 1e9


def lvt_gflop_per_clip(cfg: dict, T: int = 16, N: int = 256) -> float:
    """LvT video side: vision encoder + auxiliary encoder (GEMMs + attention over all T*N tokens)
    + the pooler FLOPs this build executes (logits and weighted sum, 4*tok*D*heads; the
    reference's K/V projections of the tokens, 16*tok*D^2, are eliminated algebraically)."""
    D, F, La = cfg["model_dim"], cfg["mlp_dim"], cfg["num_auxiliary_layers"]
    tok = T * N
    aux = (8 * D * D + 4 * D * F) * tok * La + 4 * tok * tok * D * La
    pool = 4 * tok * D * cfg["num_heads"]
    return gflop_per_clip(cfg, T, N) + (aux + pool) / 1e9


def text_gflop_per_query(cfg: dict, L: int = 64) -> float:
    D = cfg["model_dim"]
    tok = L + 1
    return ((8 * D * D + 16 * D * D) * tok + 4 * tok * tok * D) * cfg["num_unimodal_layers"] / 1e9


WORKLOADS = {
    # name: (model name, CONFIGS key, default clips per GPU)
    "base": ("videoprism_public_v1_base", "videoprism_v1_base", 32),          # configs[1]/[3]
    "large": ("videoprism_public_v1_large", "videoprism_v1_large", 16),       # configs[2]
    "lvt_large": ("videoprism_lvt_public_v1_large", "videoprism_lvt_v1_large", 32),  # configs[4]
    "lvt_base": ("videoprism_lvt_public_v1_base", "videoprism_lvt_v1_base", 32),
}


def cpu_baseline(cfg, variables, runs: int = 5, warmups: int = 2) -> dict:
    """Oracle (NumPy fp32, TEST INFRASTRUCTURE) on one clip -- a reported baseline only.  BLAS
    threads pinned to CPU_BASELINE_THREADS (the box's CPU share per GPU); `warmups` untimed runs,
    then `runs` timed runs: value = 1 / mean, with mean +- std in the sample text (SURVEY §8(d):
    B = 1, warm-up 2, runs 5, mean +- std; about 30 s of CPU work)."""
    import numpy as np
    from threadpoolctl import threadpool_info, threadpool_limits

    from oracle import videoprism_oracle as orc
    rng = np.random.default_rng(0)
    video = rng.random((1, 16, 288, 288, 3), dtype=np.float32)
    times = []
    with threadpool_limits(limits=CPU_BASELINE_THREADS):
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
        for i in range(runs + warmups):
            t0 = time.perf_counter()
            orc.factorized_encoder(variables["params"], video, cfg, mode="f32")
            if i >= warmups:
                times.append(time.perf_counter() - t0)
    mean, std = float(np.mean(times)), float(np.std(times))
    return {"value": round(1.0 / mean, 5), "unit": "clips/s", "cores": int(threads), "kind": "port",
            "blas_threads": int(threads), "host_cpus_schedulable": len(os.sched_getaffinity(0)),
            "host_cpus_total": os.cpu_count(),
            "sample": f"1 clip [1,16,288,288,3], full {cfg.get('_name', 'model')} forward, NumPy fp32 "
                      f"oracle (oracle/videoprism_oracle.py): {warmups} warm-up + {runs} timed runs, "
                      f"{mean:.2f} +- {std:.2f} s per clip (min {min(times):.2f}, max {max(times):.2f}) "
                      f"with BLAS pinned to {threads} threads; the host exposes "
                      f"{len(os.sched_getaffinity(0))} schedulable CPUs.  For context, the reference's "
                      f"published Flax-on-CPU time is 4.54 s per LvT-B pass on an Apple M3 Pro "
                      f"(FLAX_TO_MLX_CONVERSION_GUIDE.md:408); JAX cannot run here",
            "runs_s": [round(t, 3) for t in times]}


def measured_mfma_peak(device: int, iters: int = 4_000_000, reps: int = 3, f32: bool = False) -> dict | None:
    """The bf16 MFMA rate this GPU sustains with every CU issuing back-to-back MFMAs from registers on
    random operands (tools/peak/mfma_peak.hip): TFLOP/s (median of `reps` launches of
    ~0.25 s after a warm-up launch) and the in-kernel clock, for both MFMA shapes the kernels use.
    None if the microbenchmark library is not built (it is measurement only, not the product path)."""
    import ctypes
    path = os.path.join(ROOT, "tools", "peak", "libmfma_peak.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    out = {}
    shapes = ((2, "16x16x4f32"), (3, "32x32x2f32")) if f32 else ((0, "16x16x32"), (1, "32x32x16"))
    for shape, key in shapes:
        best, med, clk, ms = (ctypes.c_double() for _ in range(4))
        rc = lib.mfma_peak_run(device, shape, iters // 4 if f32 else iters, reps, ctypes.byref(best),
                               ctypes.byref(med), ctypes.byref(clk), ctypes.byref(ms))
        if rc != 0:
            return None
        out[key] = {"tflops": round(med.value, 1), "tflops_best": round(best.value, 1),
                    "clock_ghz": round(clk.value, 3), "ms_per_launch": round(ms.value, 1)}
    return out


def load_traffic(path: str, symbol: str, workload: str, src_hash: str):
    """PMC HBM bytes per launch of kernel `symbol` from a traffic record (tools/pmc_summary.py
    --json) -- only when the record was measured on the same sources and workload."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    if t.get("src_hash") != src_hash or t.get("workload") != workload:
        return None, None
    k = t.get("kernels", {}).get(symbol)
    if not k:
        return None, None
    return k.get("hbm_bytes_per_launch"), t.get("source")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_env(rank: int, world: int, port: int, base=None) -> dict:
    """A spawned rank's environment: the launcher variables, plus HSA_ENABLE_IPC_MODE_LEGACY=0
    when the caller left it unset (the host driver supports dmabuf IPC only; without it RCCL's
    peer setup fails with 'hipIpcGetMemHandle: invalid argument').  The parent has not touched
    the GPU, so this is a fresh child's environment, not a re-exec.  An explicit value is kept."""
    env = dict(os.environ if base is None else base, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn_ranks(n: int, timeout_s: float) -> int:
    """--gpus N without a launcher: N child processes of this script (RANK/LOCAL_RANK/WORLD_SIZE/
    MASTER_ADDR/MASTER_PORT set), started before this parent touches any GPU.  All children are
    polled: the first non-zero exit (a rank that died, e.g. before the rendezvous, would leave its
    siblings blocked in it) or the overall timeout terminates the others (exact PIDs), and that
    code -- 124 for the timeout -- is returned; 0 when every rank succeeded."""
    port = _free_port()
    procs = []
    for r in range(n):
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=rank_env(r, n, port)))
    deadline = time.monotonic() + timeout_s
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = next((c for c in codes if c not in (None, 0)), None)
        if bad is not None:
            rc = bad
            print(f"bench: a rank exited with {bad}; stopping the others", file=sys.stderr)
            break
        if all(c == 0 for c in codes):
            return 0
        if time.monotonic() > deadline:
            rc = 124
            print(f"bench: ranks still running after {timeout_s:.0f} s; stopping them", file=sys.stderr)
            break
        time.sleep(0.2)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=15)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc if rc > 0 else 1


# ------------------------------------------------------------------------------------------
# the step's operations: the HIP library (GpuOps) or the CPU stand-in (StandinOps, --standin)
# ------------------------------------------------------------------------------------------
class GpuOps:
    def __init__(self, eng, native):
        self.eng, self.nat = eng, native

    def forward(self, video, out):
        self.eng.forward(video, out=out)

    def pool_l2(self, out):
        return self.nat.op_pool_l2(out)

    def encode_video(self, video):
        return self.eng.encode_video(video)[0]

    def encode_text(self, ids, pad):
        return self.eng.encode_text(ids, pad)

    def similarity(self, v, t):
        return self.nat.op_similarity(v, t)


class StandinOps:
    """CPU stand-in for the multi-process plumbing test: out[b, l, d] = cos(c_b + d / D) with c_b
    the clip's first pixel (the bench fills clip b of rank r with its global index), so every
    gathered row names the clip it came from.  Not a measurement."""

    def __init__(self, D: int):
        self.D = D

    def _emb(self, video):
        import torch
        c = video[:, 0, 0, 0, 0].double()
        return torch.cos(c[:, None] + torch.arange(self.D, dtype=torch.float64)[None, :] / self.D)

    def forward(self, video, out):
        out.copy_(self._emb(video)[:, None, :].expand_as(out))

    def pool_l2(self, out):
        m = out.double().mean(dim=1)
        return (m / m.norm(dim=1, keepdim=True)).float()

    def encode_video(self, video):
        e = self._emb(video)
        return (e / e.norm(dim=1, keepdim=True)).float()

    def encode_text(self, ids, pad):
        import torch
        e = torch.sin(ids[:, :1].double() + torch.arange(self.D, dtype=torch.float64)[None, :])
        return (e / e.norm(dim=1, keepdim=True)).float()

    def similarity(self, v, t):
        return v @ t.T


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="base", choices=sorted(WORKLOADS),
                    help="base = configs[1] (default, the headline metric); large = configs[2]; "
                         "lvt_large = configs[4] video+text")
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "f32"),
                    help="compute dtype: bf16 (the headline, fprop_dtype=bfloat16) or f32 (the reference's default)")
    ap.add_argument("--batch", type=int, default=None, help="clips per GPU")
    ap.add_argument("--queries", type=int, default=8, help="text queries (LvT workloads)")
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--no-profile", action="store_true", help="no per-kernel HIP events")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-peak", action="store_true", help="skip the measured-MFMA-peak microbenchmark")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--traffic", default=None,
                    help="PMC traffic record (default: the newest profiles/traffic_r*_<workload>.json "
                         "measured on these sources)")
    ap.add_argument("--standin", action="store_true",
                    help="CPU stand-in forward over gloo: multi-process plumbing test, no measurement")
    ap.add_argument("--spawn-timeout", type=float, default=1200.0,
                    help="seconds before self-spawned ranks are stopped (--gpus N without a launcher)")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)  # launcher tests
    ap.add_argument("--hang-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, args.spawn_timeout))
    if args.fail_rank >= 0 and int(os.environ.get("RANK", 0)) == args.fail_rank:
        sys.exit(3)  # a rank that dies before the rendezvous (tests/test_distributed_cpu.py)
    if args.hang_rank >= 0 and int(os.environ.get("RANK", 0)) == args.hang_rank:
        time.sleep(3600)  # a rank that never joins (same tests)

    from videoprism import distributed

    # the process group is CPU-side (gloo) on GPU ranks too: it carries only the rendezvous, the
    # RCCL id broadcast, the barrier and the max-over-ranks; the library's vp_comm is each rank's
    # only RCCL communicator
    rank, local_rank, world = distributed.init("gloo")
    owned = []  # the RCCL communicator, once created
    try:
        _run(args, rank, local_rank, world, owned)
    finally:
        # orderly teardown on every exit path: the RCCL communicator first (its destroy
        # synchronises with the peers), then the process group
        for c in owned:
            c.close()
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(args, rank: int, local_rank: int, world: int, owned: list) -> None:
    """The bench proper, between the process group's creation and its teardown (main)."""
    import torch

    from videoprism import _native, distributed, models, params
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    name, cfg_key, default_b = WORKLOADS[args.workload]
    lvt = args.workload.startswith("lvt")
    cfg = dict(models.CONFIGS[cfg_key])
    B, T = args.batch or default_b, args.frames
    gather = world > 1 and not args.no_allgather
    if args.standin:
        dev = torch.device("cpu")
        ops = StandinOps(cfg["model_dim"])
        video = (rank * B + torch.arange(B, dtype=torch.float32))[:, None, None, None, None].expand(
            B, T, 288, 288, 3).contiguous()
        comm, eng = None, None
        if lvt:
            cfg["vocabulary_size"] = 32000
    else:
        if world > 1 and os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY") != "0":
            # the host driver supports dmabuf IPC only: RCCL's peer setup needs the legacy mode off
            print("bench: warning: HSA_ENABLE_IPC_MODE_LEGACY is not 0; RCCL may fail with "
                  "'hipIpcGetMemHandle: invalid argument' (export HSA_ENABLE_IPC_MODE_LEGACY=0)",
                  file=sys.stderr, flush=True)
        local_dev = distributed.local_device(local_rank)
        torch.cuda.set_device(local_dev)
        dev = torch.device(f"cuda:{local_dev}")
        f32 = args.dtype == "f32"
        model = models.get_model(name, fprop_dtype=None if f32 else torch.bfloat16)
        if lvt:
            cfg["vocabulary_size"] = model.vocabulary_size
            variables = params.synthetic_params(cfg, seed=0, specs=params.clip_leaf_specs(cfg))
        else:
            variables = params.synthetic_params(cfg, seed=0)
        eng = model.engine(variables, local_dev)
        ops = GpuOps(eng, _native)
        gen = torch.Generator(device=dev).manual_seed(1000 + rank)
        video = torch.rand((B, T, 288, 288, 3), generator=gen, device=dev)
        if not f32:
            video = video.to(torch.bfloat16)
        comm = distributed.Communicator(local_dev) if gather else None
        if comm is not None:
            owned.append(comm)

    last = {}
    if lvt:
        # configs[4]: text ids randint(0, V) [Q, 64] with the second half of every other query
        # padded (models_test.py:61-69), replicated on every rank
        Q, Lt = args.queries, 64
        tgen = torch.Generator(device=dev).manual_seed(7)
        ids = torch.randint(0, cfg["vocabulary_size"], (Q, Lt), generator=tgen, device=dev,
                            dtype=torch.int32)
        tpad = torch.zeros((Q, Lt), dtype=torch.float32, device=dev)
        tpad[1::2, Lt // 2:] = 1.0

        def step():
            vemb = ops.encode_video(video)
            if gather:
                vemb = distributed.all_gather_rows(vemb, world, comm, counts=[B] * world)
            temb = ops.encode_text(ids, tpad)
            last["rows"], last["sim"] = vemb, ops.similarity(vemb, temb)
    else:
        out = torch.empty((B, T * 256, cfg["model_dim"]),
                          dtype=torch.float32 if args.standin or args.dtype == "f32" else torch.bfloat16, device=dev)

        def step():
            ops.forward(video, out)
            if gather:
                last["rows"] = distributed.all_gather_rows(ops.pool_l2(out), world, comm,
                                                           counts=[B] * world)

    sync = (lambda: None) if args.standin else torch.cuda.synchronize
    for _ in range(args.warmup):
        step()
    sync()
    launches_per_fwd = 3 + 7 * (cfg["num_spatial_layers"] + cfg["num_temporal_layers"]) + 2
    if lvt:
        launches_per_fwd += 8 * cfg["num_auxiliary_layers"] + 4 + 8 * cfg["num_unimodal_layers"] + 8
    profile = not (args.no_profile or args.standin)
    breakdown, dom_name, dom_symbol = {}, None, None
    if profile:
        # per-class breakdown from one extra profiled step outside the timed region (an event
        # pair around every launch costs the stream ~2 %); the timed region then carries events
        # around the dominant class's launches only, for the live roofline
        eng.profile_only(None)
        eng.profile_enable(launches_per_fwd + 16)
        step()
        breakdown = eng.profile_read()
        dom_name = max(breakdown.items(), key=lambda kv: kv[1]["ms"])[0]
        dom_symbol = eng.kernel_name(dom_name)
        eng.profile_only([dom_name])
        eng.profile_enable(args.steps * launches_per_fwd + 16)
    distributed.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    distributed.barrier()
    elapsed = distributed.max_over_ranks(time.perf_counter() - t0)
    prof = eng.profile_read() if profile else {}
    if profile:
        eng.profile_enable(0)

    clips = world * B * args.steps
    value = clips / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    gpc = lvt_gflop_per_clip(cfg, T) if lvt else gflop_per_clip(cfg, T)
    text_gf = text_gflop_per_query(cfg) * args.queries if lvt else 0.0

    peak_tf = PEAK_F32_TFLOPS if args.dtype == "f32" else PEAK_BF16_TFLOPS
    roofline = None
    kernel_ms = {}
    if prof:
        kernel_ms = {k: round(v["ms"], 4) for k, v in
                     sorted(breakdown.items(), key=lambda kv: -kv[1]["ms"])}
        dom = prof[dom_name]
        avg_s = dom["ms"] / dom["launches"] / 1e3
        fp = _native.source_fingerprint()
        traffic, tsrc = None, None
        # fp32 kernels have records of their own (tools/pmc_traffic.sh ... f32: workload label <workload>_f32)
        tlabel = args.workload + ("_f32" if args.dtype == "f32" else "")
        for tpath in ([args.traffic] if args.traffic else
                      sorted(glob.glob(os.path.join(ROOT, "profiles", f"traffic_r*_{tlabel}.json")),
                             reverse=True)):
            traffic, tsrc = load_traffic(tpath, dom_symbol, tlabel, fp)
            if traffic is not None:
                break
        if dom["flops"] > 0:
            ach = dom["flops"] / dom["launches"] / avg_s / 1e12
            roofline = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak_tf,
                        "unit": "TFLOP/s", "frac": round(ach / peak_tf, 4),
                        "traffic": traffic}
        else:
            ach = dom["bytes"] / dom["launches"] / avg_s / 1e9
            roofline = {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS,
                        "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": traffic}
        roofline.update({"kernel": dom_name, "kernel_symbol": dom_symbol,
                         "launches": int(dom["launches"]),
                         "avg_launch_us": round(avg_s * 1e6, 2),
                         "algorithmic_per_launch": dom["flops"] / dom["launches"] if dom["flops"]
                         else dom["bytes"] / dom["launches"],
                         "algorithmic_bytes_per_launch": dom["bytes"] / dom["launches"],
                         "traffic_source": tsrc})

    if roofline is not None and rank == 0 and not args.no_peak:
        # the spec peak beside the peak this GPU sustains (bare MFMAs from registers, all CUs, random data):
        # the GEMMs issue v_mfma_f32_16x16x32_bf16, the attention kernels v_mfma_f32_32x32x16_bf16
        f32 = args.dtype == "f32"
        pk = (measured_mfma_peak(dev.index if dev.index is not None else 0, f32=f32)
              if roofline["bound"] == "mfma" else None)
        if pk is not None:
            if f32:  # the fp32 GEMMs and attention both issue v_mfma_f32_32x32x2_f32
                shape = "32x32x2f32"
            else:
                shape = "16x16x32" if "gemm" in (dom_symbol or "") else "32x32x16"
            pm = pk[shape]["tflops"]
            roofline.update({"peak_measured": pm, "frac_measured": round(roofline["achieved"] / pm, 4),
                             "peak_measured_shape": (f"v_mfma_f32_{shape[:-3]}_f32" if f32 else
                                                     f"v_mfma_f32_{shape}_bf16"),
                             "peak_measured_clock_ghz": pk[shape]["clock_ghz"],
                             "peak_measured_all": pk,
                             "peak_measured_source": "tools/peak/mfma_peak.hip: one 256-thread workgroup per CU, "
                                                     "back-to-back MFMAs from registers, random "
                                                     f"{'fp32' if f32 else 'bf16'} operands, after the timed region; "
                                                     "median of 3 launches"})

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not lvt and not args.standin:
        cfg["_name"] = name
        cpu = cpu_baseline(cfg, variables)

    standin_check = None
    if args.standin:
        rows = last.get("rows")
        expect = StandinOps(cfg["model_dim"])
        ids_all = torch.arange(world * B, dtype=torch.float32)[:, None, None, None, None]
        ref = (expect.encode_video(ids_all) if lvt else
               expect.pool_l2(expect._emb(ids_all)[:, None, :].float()))
        standin_check = {"gathered_shape": list(rows.shape) if rows is not None else None,
                         "row_order_ok": bool(rows is not None and rows.shape == ref.shape and
                                              torch.allclose(rows, ref, atol=1e-6)),
                         "similarity_shape": list(last["sim"].shape) if "sim" in last else None,
                         "ipc_mode_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")}

    if rank == 0:
        label = {"base": "VideoPrism-Base fwd", "large": "VideoPrism-Large fwd",
                 "lvt_large": "VideoPrism-LvT-Large video+text fwd",
                 "lvt_base": "VideoPrism-LvT-Base video+text fwd"}[args.workload]
        wl = (f"{name} {args.dtype} forward, B={B} clips/GPU x {world} GPU, {T}x288x288x3"
              + (f", {args.queries} text queries x 64 tokens, gathered video_emb @ text_emb.T"
                 if lvt else "")
              + ((", gloo all-gather (stand-in)" if args.standin else
                  ", RCCL all-gather (vp_allgather) of pooled embeddings") if gather else ""))
        line = {
            "metric": f"clips/sec (16x288x288) {label}{' fp32' if args.dtype == 'f32' else ''}; % MFMA peak",
            "value": round(value, 3), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic uniform[0,1) clips generated on device; random-init weights of the "
                    "real architecture (no checkpoint offline)",
            "config": {"workload": wl,
                       "model": name, "global_batch": B * world, "frames": T,
                       "parallelism": f"dp{world} (batch-sharded clips)"},
            "mfma_util_whole_forward": round((value / world * gpc + text_gf / ms_per_step * 1e3)
                                             / 1e3 / peak_tf, 4),
            "gflop_per_clip": round(gpc, 2),
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernel_ms_per_step": kernel_ms,
            "kernel_ms_per_step_source": "HIP events around every launch of one extra step after "
                                         "warmup (outside the timed region)",
        }
        if args.standin:
            line.update({"data": "CPU stand-in forward (--standin): plumbing test, not a measurement",
                         "dtype": "f32", "standin_check": standin_check})
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
