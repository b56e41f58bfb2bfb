"""Bitwise A/B of whole forwards between this tree and another revision (tools/ab_build.sh): run once
per tree, each run prints one JSON line of output hashes; equal lines = bitwise-equal outputs.

  python tools/ab_forward_hash.py [TREE_ROOT]        # default: this tree

The model, weights and inputs are built from seeds inside the run, so both trees see the same
inputs.  Covered: Base full depth T = 16 bf16 (the bench's path), Base 2+1 layers at T = 8 / 20 /
32 in bf16 and fp32 (precomputed temporal tables and the generic temporal attention), Large 1+1
layers at T = 16 bf16 (8 -> 16 temporal interpolation), LvT-Base reduced depth at 288 x 288, T = 4 / 16
(auxiliary attention over 1024 / 4096 tokens) in bf16 and fp32: video, frame and text embeddings.
"""
import hashlib
import json
import os
import sys

root = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.dirname(__file__)))
sys.path[:0] = [root, os.path.join(root, "videoprism-mlx_amd")]

import torch  # noqa: E402

from videoprism import encoders, models, params  # noqa: E402


def run(cfg, T, bf16, B=2, seed=0):
    var = params.synthetic_params(cfg, seed=seed)
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedEncoder(**cfg),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    g = torch.Generator(device="cuda").manual_seed(seed + T)
    video = torch.rand((B, T, 288, 288, 3), generator=g, device="cuda")
    if bf16:
        video = video.to(torch.bfloat16)
    emb, _ = m.apply(var, video)
    torch.cuda.synchronize()
    return hashlib.sha256(emb.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]


out = {"tree": root}
base = dict(models.CONFIGS["videoprism_v1_base"])
out["base_full_t16_bf16"] = run(base, 16, True)
small = dict(base, num_spatial_layers=2, num_temporal_layers=1)
for T in (8, 20, 32):
    for bf16 in (False, True):
        out[f"base21_t{T}_{'bf16' if bf16 else 'f32'}"] = run(small, T, bf16)
large = dict(models.CONFIGS["videoprism_v1_large"], num_spatial_layers=1, num_temporal_layers=1)
out["large11_t16_bf16"] = run(large, 16, True)


def run_lvt(T, bf16, B=2, seed=3):
    """LvT-Base (1+1 vision, 2 auxiliary, 2 text layers) at 288 x 288: video, frame and text embeddings."""
    cfg = dict(models.CONFIGS["videoprism_lvt_v1_base"], vocabulary_size=1000, num_spatial_layers=1,
               num_temporal_layers=1, num_unimodal_layers=2)
    var = params.synthetic_params(cfg, seed=seed, specs=params.clip_leaf_specs(cfg))
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**cfg),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    eng = m.engine(var, torch.cuda.current_device())
    g = torch.Generator(device="cuda").manual_seed(seed + T)
    video = torch.rand((B, T, 288, 288, 3), generator=g, device="cuda")
    ids = torch.randint(0, 1000, (3, 16), generator=g, device="cuda", dtype=torch.int32)
    pads = torch.zeros((3, 16), device="cuda")
    pads[0, 8:] = 1.0
    v, f, _, _ = eng.encode_video(video.to(torch.bfloat16) if bf16 else video, want_frames=True)
    t = eng.encode_text(ids, pads)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for a in (v, f, t):
        h.update(a.contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return h.hexdigest()[:16]


for T in (4, 16):
    for bf16 in (False, True):
        out[f"lvt_base_t{T}_{'bf16' if bf16 else 'f32'}"] = run_lvt(T, bf16)
print(json.dumps(out))
