"""Parity report in the shape of the reference's verify_clip_models.py: for each LvT model, run this
library (HIP, MI355X) and the NumPy oracle (oracle/videoprism_oracle.py, fp64) on the same inputs
and print max / mean absolute differences of the video and text embeddings and of their cosine
similarity, then PASS when every max difference is within the tolerance.

The reference compares its Flax and MLX paths on real weights and a decoded video; neither JAX nor
the checkpoints exist offline, so here the weights are synthetic (params.synthetic_params), the clip
is uniform[0,1) and the token ids deterministic.  --layers reduces every stack (the fp64 oracle of
the full models takes minutes on the CPU).

    python tools/verify_clip_models.py --layers 1
    python tools/verify_clip_models.py --models videoprism_lvt_public_v1_base --frames 8
"""

from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]


def verify(model_name: str, args) -> bool:
    import torch

    from oracle import videoprism_oracle as orc
    from videoprism import encoders, models, params

    print(f"\n{'=' * 80}\nTesting: {model_name}\n{'=' * 80}")
    print("\n[1/3] Loading models...")
    cfg = dict(models.CONFIGS[model_name.replace("_public", "")])
    cfg.setdefault("vocabulary_size", args.vocab)
    if args.layers:
        cfg.update(num_spatial_layers=args.layers, num_temporal_layers=min(args.layers, 4),
                   num_auxiliary_layers=min(args.layers, 2), num_unimodal_layers=args.layers)
    variables = params.synthetic_params(cfg, seed=0, specs=params.clip_leaf_specs(cfg))
    dt = torch.bfloat16 if args.dtype == "bf16" else None
    model = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**cfg), fprop_dtype=dt)
    print("[2/3] Loading video and text...")
    rng = np.random.default_rng(0)
    video = rng.random((1, args.frames, 288, 288, 3), dtype=np.float32)
    ids = rng.integers(0, cfg["vocabulary_size"], (3, 64)).astype(np.int32)
    pads = np.zeros((3, 64), np.float32)
    pads[1::2, 32:] = 1.0
    print("[3/3] Running inference...")
    v, t, _ = model.apply(variables, video, ids, pads)
    rv, rt, _ = orc.video_clip(variables["params"], cfg, video, ids, pads, "f64")
    v, t = np.asarray(v, np.float64), np.asarray(t, np.float64)
    vd, td = np.abs(v - rv), np.abs(t - rt)
    sim, rsim = v @ t.T, rv @ rt.T
    print("\n  Comparison Results:\n  " + "-" * 76)
    print(f"  Video embeddings:\n    Max diff:  {vd.max():.6e}\n    Mean diff: {vd.mean():.6e}")
    print(f"  Text embeddings:\n    Max diff:  {td.max():.6e}\n    Mean diff: {td.mean():.6e}")
    print(f"  Cosine similarity (clip vs each query):\n    oracle: {np.round(rsim[0], 6).tolist()}\n"
          f"    HIP:    {np.round(sim[0], 6).tolist()}\n    Max diff: {np.abs(sim - rsim).max():.6e}")
    tol = args.tol if args.tol else (1e-3 if args.dtype == "bf16" else 1e-5)
    ok = max(vd.max(), td.max(), np.abs(sim - rsim).max()) <= tol
    print(f"  {'PASS' if ok else 'FAIL'} - max differences {'within' if ok else 'above'} {tol:g}")
    return ok


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--models", nargs="+", default=["videoprism_lvt_public_v1_base", "videoprism_lvt_public_v1_large"])
    ap.add_argument("--layers", type=int, default=1, help="depth of every stack (0: the full model)")
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--tol", type=float, default=0.0, help="default 1e-3 (bf16) / 1e-5 (fp32), north_star bars")
    args = ap.parse_args()
    print("=" * 80 + "\nVerifying CLIP Models: HIP (MI355X) vs NumPy oracle (fp64)\n" + "=" * 80)
    results = [verify(m, args) for m in args.models]
    print("\n" + "=" * 80 + "\nVerification Complete\n" + "=" * 80)
    sys.exit(0 if all(results) else 1)


if __name__ == "__main__":
    main()
