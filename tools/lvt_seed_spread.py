"""Spread of the full-depth LvT-Base bf16 video-embedding error over clips (the case that decides the 1e-3
bar of tests/test_gpu_clip.py::test_clip_full_lvt_base_bf16 at seed 11): for each seed, the same construction
as that test (synthetic parameters and frames of the seed, B = 1, T = 8, two 64-token texts), the GPU bf16
path against the fp64 oracle, and the cast floor (the oracle in fp64 on bf16-rounded parameters and frames,
`wbf16`).  The oracle results are cached (--cache) so another build of the library (a tools/ab_build.sh tree,
run with --root) is compared on the same references.

  python tools/lvt_seed_spread.py --seeds 11 12 13 14 15 16 --cache gpurun_out/lvt_oracle.npz [--label exact]
"""
import argparse
import os
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument("--seeds", type=int, nargs="+", default=[11, 12, 13, 14])
ap.add_argument("--cache", default="gpurun_out/lvt_oracle.npz")
ap.add_argument("--root", default=None, help="tree whose library to load (default: this one)")
ap.add_argument("--label", default="this")
ap.add_argument("--oracle-only", action="store_true")
args = ap.parse_args()
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOT = os.path.abspath(args.root) if args.root else HERE
sys.path[:0] = [HERE, os.path.join(ROOT, "videoprism-mlx_amd")]
import numpy as np  # noqa: E402

from oracle import videoprism_oracle as orc  # noqa: E402
from videoprism import encoders, models, params  # noqa: E402


def cfg_lvt_base():
    c = dict(models.CONFIGS["videoprism_lvt_v1_base"])
    c["vocabulary_size"] = 1000
    return c


def inputs(cfg, seed):
    var = params.synthetic_params(cfg, seed, specs=params.clip_leaf_specs(cfg))
    video = np.random.default_rng(seed).random((1, 8, 288, 288, 3), dtype=np.float32)
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, cfg["vocabulary_size"], (2, 64)).astype(np.int32)
    pads = np.zeros((2, 64), np.float32)
    pads[0, 32:] = 1.0
    return var, video, ids, pads


def bf16_round(a):
    a = np.ascontiguousarray(a, np.float32)
    u = a.view(np.uint32)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32)


def main():
    cfg = cfg_lvt_base()
    cache = dict(np.load(args.cache)) if os.path.exists(args.cache) else {}
    rows = []
    for seed in args.seeds:
        var, video, ids, pads = inputs(cfg, seed)
        if f"f64_{seed}" not in cache:
            t0 = time.time()
            rv, _, _ = orc.video_clip(var["params"], cfg, video, None, None, "f64")
            cache[f"f64_{seed}"] = rv
            cast, _, _ = orc.video_clip(var["params"], cfg, bf16_round(video), None, None, "wbf16")
            cache[f"cast_{seed}"] = cast
            np.savez(args.cache, **cache)
            print(f"seed {seed}: oracle {time.time() - t0:.0f} s", flush=True)
        if args.oracle_only:
            continue
        import torch
        m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**cfg), fprop_dtype=torch.bfloat16)
        eng = m.engine(var, torch.cuda.current_device())
        x = torch.from_numpy(video).cuda().to(torch.bfloat16)
        vemb = eng.encode_video(x)[0]
        torch.cuda.synchronize()
        v = vemb.cpu().numpy().astype(np.float64)
        ref, cast = cache[f"f64_{seed}"], cache[f"cast_{seed}"]
        e, c = float(np.abs(v - ref).max()), float(np.abs(cast - ref).max())
        rows.append((seed, e, c))
        print(f"{args.label} seed {seed}: video embedding max-abs vs fp64 {e:.3e} (cast floor {c:.3e})", flush=True)
    if rows:
        e = np.array([r[1] for r in rows])
        c = np.array([r[2] for r in rows])
        print(f"{args.label}: over {len(rows)} clips mean {e.mean():.3e} median {np.median(e):.3e} max {e.max():.3e}; "
              f"cast floor mean {c.mean():.3e} max {c.max():.3e}", flush=True)


if __name__ == "__main__":
    main()
