"""Forward-pass timing harness in the shape of the reference's scripts/benchmark_performance.py:
per-run wall-clock timings after warm-up, mean / std / min / max, and the peak resident-set size.

The reference times its Flax and MLX forwards of the LvT video-text model on a decoded video and
tokenized text.  Here the frameworks are this library on the MI355X ("hip", device-synchronised)
and the NumPy CPU restatement ("oracle", oracle/videoprism_oracle.py -- test infrastructure, used
here only as the CPU point of comparison); video decoding and the SentencePiece tokenizer are out of
scope, so the clip is synthetic uniform[0,1) (or a saved [T,H,W,3] array via --video-npy) and the
text queries are deterministic token ids with the reference tests' padding pattern.

    python tools/benchmark_performance.py --framework both --runs 20 --warmup 3
    python tools/benchmark_performance.py --framework hip --model-name videoprism_public_v1_base
"""

from __future__ import annotations

import argparse
import os
import resource
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]

DEFAULT_MODEL_NAME = "videoprism_lvt_public_v1_base"


def _summary(durations: list[float]) -> str:
    """One line over the timed runs: count, median and spread in milliseconds (empty -> note)."""
    if len(durations) == 0:
        return "no timed runs"
    ms = np.asarray(durations, dtype=np.float64) * 1e3
    lo, med, hi = np.percentile(ms, [0, 50, 100])
    return f"n={ms.size} median {med:.1f} ms (range {lo:.1f}-{hi:.1f} ms, sd {ms.std():.1f} ms)"


def _rss_gb() -> float:
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / (1024 ** 2)  # Linux: KiB


def _inputs(args, cfg):
    rng = np.random.default_rng(0)
    if args.video_npy:
        video = np.load(args.video_npy)[None].astype(np.float32)  # [1, T, H, W, 3] in [0, 1]
    else:
        video = rng.random((args.batch, args.num_frames, args.target_size, args.target_size, 3), dtype=np.float32)
    q = len(args.text_queries.split("||"))
    vocab = cfg.get("vocabulary_size", 32000)
    ids = rng.integers(0, vocab, (q, 64)).astype(np.int32)
    pads = np.zeros((q, 64), np.float32)
    pads[1::2, 32:] = 1.0  # models_test.py:61-69 pattern
    return video, ids, pads


def _model(args):
    import torch

    from videoprism import models, params
    key = args.model_name.replace("_public", "")  # videoprism_lvt_public_v1_base -> videoprism_lvt_v1_base
    cfg = dict(models.CONFIGS[key])
    lvt = "lvt" in args.model_name
    if lvt:
        cfg.setdefault("vocabulary_size", 32000)  # models.py text-tokenizer vocabulary
    if args.layers:
        cfg.update(num_spatial_layers=args.layers, num_temporal_layers=min(args.layers, cfg["num_temporal_layers"]))
        if lvt:
            cfg.update(num_unimodal_layers=args.layers, num_auxiliary_layers=min(args.layers, 2))
    specs = params.clip_leaf_specs(cfg) if lvt else None
    variables = params.synthetic_params(cfg, seed=0, specs=specs) if lvt else params.synthetic_params(cfg, seed=0)
    return cfg, lvt, variables, torch


def benchmark_hip(args):
    from videoprism import encoders, models
    print("\n=== HIP (MI355X) benchmark ===")
    cfg, lvt, variables, torch = _model(args)
    dt = torch.bfloat16 if args.dtype == "bf16" else None
    fn = encoders.FactorizedVideoCLIP if lvt else encoders.FactorizedEncoder
    model = models.get_model(None, model_fn=lambda: fn(**cfg), fprop_dtype=dt)
    video, ids, pads = _inputs(args, cfg)
    dev = torch.device("cuda:0")
    v = torch.from_numpy(video).to(dev)
    if dt is not None:
        v = v.to(dt)
    tids, tpads = torch.from_numpy(ids).to(dev), torch.from_numpy(pads).to(dev)

    def run_once():
        t0 = time.perf_counter()
        if lvt:
            model.apply(variables, v, tids, tpads, normalize=args.normalize)
        else:
            model.apply(variables, v)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    for _ in range(args.warmup):
        run_once()
    durations = [run_once() for _ in range(args.runs)]
    print("runs:", args.runs, " warmup:", args.warmup)
    print("timings:", [f"{t:.4f}" for t in durations])
    print("timing:", _summary(durations))
    print(f"ru_maxrss: {_rss_gb():.3f} GB")


def benchmark_oracle(args):
    from oracle import videoprism_oracle as orc
    print("\n=== NumPy CPU restatement (oracle) benchmark ===")
    cfg, lvt, variables, _ = _model(args)
    video, ids, pads = _inputs(args, cfg)
    mode = "f32"

    def run_once():
        t0 = time.perf_counter()
        if lvt:
            orc.video_clip(variables["params"], cfg, video, ids, pads, mode)
        else:
            orc.factorized_encoder(variables["params"], video, cfg, mode=mode)
        return time.perf_counter() - t0

    for _ in range(args.oracle_warmup):
        run_once()
    durations = [run_once() for _ in range(args.oracle_runs)]
    print("runs:", args.oracle_runs, " warmup:", args.oracle_warmup)
    print("timings:", [f"{t:.4f}" for t in durations])
    print("timing:", _summary(durations))
    print(f"ru_maxrss: {_rss_gb():.3f} GB")


def main():
    parser = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    parser.add_argument("--framework", choices=["hip", "oracle", "both"], default="both")
    parser.add_argument("--model-name", default=DEFAULT_MODEL_NAME)
    parser.add_argument("--video-npy", default=None, help="[T,H,W,3] float array in [0,1] (decoded frames)")
    parser.add_argument("--num-frames", type=int, default=16)
    parser.add_argument("--target-size", type=int, default=288)
    parser.add_argument("--batch", type=int, default=1)
    parser.add_argument("--text-queries", default="a person walking||drumming on water bottles||a car driving",
                        help="pipe-delimited prompts; only their count is used (no tokenizer offline)")
    parser.add_argument("--runs", type=int, default=20)
    parser.add_argument("--warmup", type=int, default=3)
    parser.add_argument("--oracle-runs", type=int, default=2)
    parser.add_argument("--oracle-warmup", type=int, default=0)
    parser.add_argument("--dtype", choices=["bf16", "f32"], default="bf16", help="HIP fprop dtype")
    parser.add_argument("--layers", type=int, default=0, help="reduce every stack to this depth (0: full)")
    parser.add_argument("--normalize", action="store_true", help="Return normalized embeddings.")
    args = parser.parse_args()
    if args.framework in {"hip", "both"}:
        benchmark_hip(args)
    if args.framework in {"oracle", "both"}:
        benchmark_oracle(args)


if __name__ == "__main__":
    main()
