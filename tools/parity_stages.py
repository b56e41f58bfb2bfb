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


def base_stages(args):
    """Full Base, B=1, T=8, normal(0, 0.1) frames (tests/test_gpu_encoder.py
    test_full_base_b1_bf16_vs_oracle): the build-defined pooled vector (token mean + L2) split into the
    spatial half (GPU spatial_features vs fp64) and the temporal half (the oracle's fp64 temporal stack
    replayed from the GPU's spatial features)."""
    import torch

    from oracle import videoprism_oracle as orc
    from videoprism import models, params
    cfg = models.CONFIGS["videoprism_v1_base"]
    var = params.synthetic_params(cfg, seed=0)
    video = np.random.default_rng(9).normal(0.0, 0.1, (1, 8, 288, 288, 3)).astype(np.float32)
    mdl = models.get_model("videoprism_public_v1_base", fprop_dtype=torch.bfloat16)
    emb, out = mdl.apply(var, video, train=False, return_intermediate=["spatial_features"])
    p = var["params"]
    ref, rout = orc.factorized_encoder(p, video, cfg, mode="f64", return_intermediate=["spatial_features"])
    emu, _ = orc.factorized_encoder(p, video, cfg, mode="bf16")
    wq, _ = orc.factorized_encoder(p, orc.round_bf16(video), cfg, mode="wbf16")

    def pool(e):
        m = np.asarray(e, np.float64).mean(axis=1)
        return m / np.sqrt((m * m).sum(-1, keepdims=True) + 1e-12)

    # temporal half of factorized_encoder (oracle lines after spatial_ln), from given spatial features
    def temporal_from(spf):
        nm = orc.Numerics("f64")
        b, t, n, D = 1, 8, 256, cfg["model_dim"]
        f = np.asarray(spf, np.float64).reshape(b, t, n, D).transpose(0, 2, 1, 3).reshape(b * n, t, D)
        t_emb = np.asarray(p["temporal_pos_emb"]["emb_var"], np.float64)[:cfg["pos_emb_shape"][0]][None]
        if t_emb.shape[1] != t:
            t_emb = orc.interpolate_emb_1d(t_emb, t)
        f = f + t_emb
        f = orc.stacked_transformer(f, None, p["temporal_encoder"]["transformers_stack"], nm,
                                    cfg["num_temporal_layers"], cfg["num_heads"], cfg.get("atten_logit_cap", 0.0))
        f = orc.layer_norm(f, p["temporal_ln"]["scale"], p["temporal_ln"]["bias"], nm)
        return f.reshape(b, n, t, D).transpose(0, 2, 1, 3).reshape(b, t * n, D)

    rep = temporal_from(out["spatial_features"])
    sp_err = np.abs(np.asarray(out["spatial_features"], np.float64) - rout["spatial_features"])
    rec = {
        "model": "videoprism_v1_base", "frames": 8,
        "pooled_vs_f64": float(np.abs(pool(emb) - pool(ref)).max()),
        "reference_bf16_emulation_pooled_vs_f64": float(np.abs(pool(emu) - pool(ref)).max()),
        "bf16_params_and_frames_only_pooled_vs_f64": float(np.abs(pool(wq) - pool(ref)).max()),
        "pooled_vs_bf16_params_oracle": float(np.abs(pool(emb) - pool(wq)).max()),
        "spatial_features": {"max": float(sp_err.max()), "mean": float(sp_err.mean())},
        "pooled_from_gpu_spatial_vs_f64": float(np.abs(pool(rep) - pool(ref)).max()),
        "pooled_gpu_vs_replay": float(np.abs(pool(emb) - pool(rep)).max()),
        "tokens_vs_f64": {"max": float(np.abs(emb - ref).max()), "mean": float(np.abs(emb - ref).mean())},
    }
    print(json.dumps(rec, indent=1), flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="videoprism_lvt_v1_base")
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--json", default=None)
    ap.add_argument("--base", action="store_true", help="the FactorizedEncoder Base T=8 pooled case instead")
    args = ap.parse_args()
    if args.base:
        rec = base_stages(args)
        if args.json:
            with open(args.json, "w") as f:
                json.dump(rec, f, indent=1)
        return

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
    # fp64 arithmetic on the bf16-rounded parameters and frames: what the bf16 mode's parameter / input
    # cast alone costs (the floor any bf16 implementation of the reference shares)
    rv_w, _, _ = orc.video_clip(p, cfg, orc.round_bf16(video), mode="wbf16")

    def mx(a, b):
        return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())

    tok_err = np.abs(st_gpu - st_ref)
    rec = {
        "model": args.model, "frames": args.frames, "seed": args.seed,
        "video_emb_vs_f64": mx(v_gpu, rv),
        "reference_bf16_emulation_vs_f64": mx(rv_bf, rv),
        "bf16_params_and_frames_only_vs_f64": mx(rv_w, rv),
        "video_emb_vs_bf16_params_oracle": mx(v_gpu, rv_w),
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
