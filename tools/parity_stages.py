"""Where the bf16 error of the LvT video embedding comes from, on the GPU box:

    python tools/parity_stages.py [--model videoprism_lvt_v1_base] [--frames 8] [--seed 11]

Runs the full-depth LvT model in bf16 on one clip (the case of tests/test_gpu_clip.py
test_clip_full_lvt_base_bf16) and the fp64 oracle, and splits the embedding's max-abs error vs
fp64 into stages by replaying the oracle from the GPU's own intermediates:

  vision     GPU spatio-temporal tokens vs the oracle's (per-token max / mean, relative)
  from_vis   the oracle's fp64 auxiliary encoder + pooler + L2 fed with the GPU's tokens, vs fp64:
             the part of the final error the vision encoder's tokens carry
  after_vis  the GPU's embedding vs that replay: the part the GPU's auxiliary encoder, pooler and
             normalisation add
and the same split inside the pooler (pre-LayerNorm pooled vector, LayerNorm output) from the
oracle replay.  Oracle = test infrastructure (oracle/), used here as the checker only."""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]


def rest_of_video_path(params, cfg, feats, nm):
    """encoders.py:846-866 from the spatio-temporal tokens: auxiliary encoder, contrastive pooler
    (pre-LN vector and LN output kept), L2 normalisation -- the oracle's own functions."""
    from oracle import videoprism_oracle as orc
    D, heads = cfg["model_dim"], cfg["num_heads"]
    cap = cfg.get("atten_logit_cap", 0.0)
    x = feats
    if cfg.get("num_auxiliary_layers", 0) > 0:
        x = orc.stacked_transformer_causal(x, None, params["auxiliary_encoder"]["transformers_stack"], nm,
                                           cfg["num_auxiliary_layers"], heads, cap, False, orc.gelu)
    p = params["contrastive_vision_pooler"]
    pooled_ln = orc.atten_token_pooling(x, p, nm, heads, 4 * D)[:, 0]
    return x, pooled_ln, orc.l2_normalize(pooled_ln)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="videoprism_lvt_v1_base")
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()

    import torch

    from oracle import videoprism_oracle as orc
    from videoprism import encoders, models, params

    cfg = dict(models.CONFIGS[args.model])
    cfg["vocabulary_size"] = 1000
    var = params.synthetic_params(cfg, args.seed, specs=params.clip_leaf_specs(cfg))
    video = np.random.default_rng(args.seed).random((1, args.frames, 288, 288, 3), dtype=np.float32)
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**cfg), fprop_dtype=torch.bfloat16)
    eng = m.engine(var, torch.cuda.current_device())
    vemb, _, _, st = eng.encode_video(torch.from_numpy(video).cuda().to(torch.bfloat16), want_spatiotemporal=True)
    torch.cuda.synchronize()
    v_gpu = vemb.double().cpu().numpy()
    st_gpu = st.double().cpu().numpy()

    p = var["params"]
    rv, _, rout = orc.video_clip(p, cfg, video, mode="f64", return_intermediate=("spatiotemporal_features",))
    st_ref = rout["spatiotemporal_features"]
    nm = orc.Numerics("f64")
    aux_ref, pooled_ref, _ = rest_of_video_path(p, cfg, st_ref, nm)
    aux_rep, pooled_rep, v_rep = rest_of_video_path(p, cfg, st_gpu, nm)
    # the oracle's emulation of the reference's own bf16 graph, for scale
    rv_bf, _, _ = orc.video_clip(p, cfg, video, mode="bf16")

    def mx(a, b):
        return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())

    tok_err = np.abs(st_gpu - st_ref)
    rec = {
        "model": args.model, "frames": args.frames, "seed": args.seed,
        "video_emb_vs_f64": mx(v_gpu, rv),
        "reference_bf16_emulation_vs_f64": mx(rv_bf, rv),
        "vision_tokens": {"max": float(tok_err.max()), "mean": float(tok_err.mean()),
                          "rel_rms": float(np.sqrt((tok_err ** 2).mean() / (st_ref ** 2).mean()))},
        "aux_tokens_from_gpu_vision": {"max": mx(aux_rep, aux_ref),
                                       "rel_rms": float(np.sqrt(((aux_rep - aux_ref) ** 2).mean()
                                                                / (aux_ref ** 2).mean()))},
        "pooled_ln_from_gpu_vision": mx(pooled_rep, pooled_ref),
        "video_emb_from_gpu_vision": mx(v_rep, rv),
        "video_emb_gpu_vs_replay": mx(v_gpu, v_rep),
        "pooled_ln_norm": float(np.linalg.norm(pooled_ref)),
    }
    print(json.dumps(rec, indent=1), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
