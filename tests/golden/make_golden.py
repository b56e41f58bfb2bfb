"""Generates the committed golden fixtures from the NumPy oracle (oracle/videoprism_oracle.py).

PARITY UNPINNED by the reference: its tests hold no value-level vectors for this path
(SURVEY.md §8(c)), JAX is not installed here, so these fixtures pin the oracle against
future drift and give the GPU tests fixed vectors; their cross-check is the independent
torch restatement (tests/torch_restatement.py) and the structural pins of the reference
tests.  Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]

from oracle import videoprism_oracle as orc  # noqa: E402
from videoprism import models, params  # noqa: E402

# encoders_test.py:130,145-156 — the reference's own tiny FactorizedEncoder
TINY = dict(patch_size=4, pos_emb_shape=(16, 16, 16), model_dim=8, num_spatial_layers=2,
            num_temporal_layers=2, num_heads=2, mlp_dim=4, atten_logit_cap=50.0)


def g1_tiny():
    var = params.synthetic_params(TINY, seed=0)
    flat = params.flatten(var["params"])
    x = np.random.default_rng(0).normal(0.0, 0.1, (1, 4, 16, 16, 3)).astype(np.float32)
    emb, out = orc.factorized_encoder(var["params"], x, TINY, "f64", return_intermediate=True)
    fp = np.zeros((1, 4), np.float32)
    fp[:, 2:] = 1.0  # encoders_test.py:138-142
    emb_p, _ = orc.factorized_encoder(var["params"], x, TINY, "f64", frame_paddings=fp)
    arrays = {f"param/{k}": v for k, v in flat.items()}
    arrays.update(inputs=x, frame_paddings=fp, embeddings=emb, spatial_features=out["spatial_features"],
                  embeddings_padded=emb_p)
    np.savez_compressed(os.path.join(HERE, "g1_tiny.npz"), **arrays)


def g2_base_dims():
    cfg = dict(models.CONFIGS["videoprism_v1_base"])
    cfg.update(num_spatial_layers=2, num_temporal_layers=1)
    var = params.synthetic_params(cfg, seed=1)
    flat = params.flatten(var["params"])
    x = np.random.default_rng(3).random((1, 2, 288, 288, 3), dtype=np.float32)
    emb, _ = orc.factorized_encoder(var["params"], x, cfg, "f64")
    idx = np.arange(0, emb.size, 997)
    np.savez_compressed(
        os.path.join(HERE, "g2_base_dims.npz"),
        param_names=np.array(sorted(flat)),
        param_sums=np.array([float(np.sum(flat[k], dtype=np.float64)) for k in sorted(flat)]),
        param_heads=np.stack([flat[k].ravel()[:4] for k in sorted(flat)]),
        input_seed=np.array(3), param_seed=np.array(1), sample_index=idx,
        sample_values=emb.ravel()[idx], row_sums=emb.sum(axis=-1).ravel(),
        shape=np.array(emb.shape))


def g4_ops():
    rng = np.random.default_rng(4)
    nm = orc.Numerics("f64")
    x = rng.normal(1.0, 3.0, (5, 768))
    sc, bi = rng.normal(0, 0.1, 768), rng.normal(0, 0.1, 768)
    g = np.linspace(-6, 6, 97)
    q, k, v = rng.normal(0, 1, (3, 2, 16, 64))
    q = q * 4.0
    kp = np.zeros((2, 16))
    kp[1, ::3] = 1
    img = rng.random((2, 6, 6, 3))
    np.savez_compressed(
        os.path.join(HERE, "g4_ops.npz"),
        ln_x=x, ln_scale=sc, ln_bias=bi, ln_out=orc.layer_norm(x, sc, bi, nm),
        gelu_x=g, gelu_y=orc.gelu(g),
        att_q=q, att_k=k, att_v=v, att_key_pad=kp,
        att_out=orc.capped_softmax_attention(q, k, v, 50.0, kp),
        patch_img=img, patch_out=orc.image_to_patch(img, 3),
        resize_up_8_16=orc._resize_weights(8, 16), resize_down_16_4=orc._resize_weights(16, 4))


# encoders_test.py:290-324 — the reference's own tiny FactorizedVideoCLIP
CLIP_TINY = dict(patch_size=4, pos_emb_shape=(16, 16, 16), num_spatial_layers=2, num_temporal_layers=2,
                 mlp_dim=4, num_auxiliary_layers=1, vocabulary_size=20, enable_causal_atten=True,
                 num_unimodal_layers=2, model_dim=8, num_heads=2, atten_logit_cap=50.0)


def g5_clip_tiny():
    cfg = CLIP_TINY
    var = params.synthetic_params(cfg, seed=5, specs=params.clip_leaf_specs(cfg))
    flat = params.flatten(var["params"])
    rng = np.random.default_rng(5)
    x = rng.normal(0.0, 0.1, (1, 4, 16, 16, 3)).astype(np.float32)
    ids = rng.integers(0, 20, (1, 10)).astype(np.int32)
    pads = np.zeros((1, 10), np.float32)
    pads[:, 5:] = 1.0  # encoders_test.py:304-305
    v, t, out = orc.video_clip(var["params"], cfg, x, ids, pads, "f64", return_intermediate=True)
    arrays = {f"param/{k}": a for k, a in flat.items()}
    arrays.update(inputs=x, text_token_ids=ids, text_paddings=pads, video_embeddings=v, text_embeddings=t,
                  frame_embeddings=out["frame_embeddings"],
                  spatiotemporal_features=out["spatiotemporal_features"])
    np.savez_compressed(os.path.join(HERE, "g5_clip_tiny.npz"), **arrays)


# full-depth models at the metric's clip length (configs[1] / configs[2]): the oracle in fp64 and
# in its emulation of the reference's bf16 graph, on clip 0 of the GPU tests' batches.  Stored:
# the L2-normalised token-mean ("pooled") vector, every 64th token row, and the inputs' seeds
# (the GPU tests regenerate the identical video and weights from them).
FULL = {"g6_base_t16": ("videoprism_v1_base", 0, 11), "g7_large_t16": ("videoprism_v1_large", 0, 12)}


def full_video(seed, T=16):
    return np.random.default_rng(seed).random((1, T, 288, 288, 3), dtype=np.float32)


def g_full(tag, T=16, modes=("f64", "bf16")):
    name, pseed, vseed = FULL[tag]
    cfg = models.CONFIGS[name]
    var = params.synthetic_params(cfg, seed=pseed)
    x = full_video(vseed, T)
    arrays = dict(param_seed=np.array(pseed), video_seed=np.array(vseed), model=np.array(name), T=np.array(T))
    for mode in modes:
        e, _ = orc.factorized_encoder(var["params"], x, cfg, mode)
        m = e.astype(np.float64).mean(axis=1)
        arrays[f"pooled_{mode}"] = m / np.sqrt((m * m).sum(-1, keepdims=True) + 1e-12)
        # fp64 rows for the fp32 bar (1e-5); float32 storage would round them by up to ~1e-7 * |y|
        arrays[f"rows_{mode}"] = e[0, ::64].astype(np.float64 if T > 16 else np.float32)
        arrays[f"frame_mean_{mode}"] = e[0].reshape(T, -1, e.shape[-1]).mean(axis=1).astype(np.float32)
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **arrays)


# Clips longer than the temporal table (encoders.py:543-553 interpolates the
# temporal pos-emb to any T): full-depth Base at T = 48 / 64 (16 -> 48 / 64) and Large at T = 48
# (8 -> 48), fp64 only (the bf16 bars are the pooled vector and the token mean-abs)
LONG = {"g9_base_t48": ("videoprism_v1_base", 0, 21, 48), "g10_base_t64": ("videoprism_v1_base", 0, 22, 64),
        "g11_large_t48": ("videoprism_v1_large", 0, 23, 48)}
FULL.update({k: v[:3] for k, v in LONG.items()})


# configs[4]'s per-rank workload at full depth: FactorizedVideoCLIP with videoprism_lvt_v1_large
# (24 + 4 vision layers, 2 auxiliary layers over all 4096 tokens, 12 text layers; encoders.py:762-910,
# models.py:131-145), B = 1 clip of T = 16 frames, two 64-token texts with the second half of one
# padded (models_test.py:61-69).  Stored: the video / text embeddings and their similarity
# (README.md:81) from the fp64 oracle and from its emulation of the reference's bf16 graph, plus
# the frame embeddings; the GPU tests regenerate weights, video and ids from the stored seeds.
G8 = dict(cfg="videoprism_lvt_v1_large", vocabulary_size=32000, param_seed=8, video_seed=18, text_seed=28,
          Q=2, L=64)


def g8_text(seed, Q, L, V):
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, V, (Q, L)).astype(np.int32)
    pads = np.zeros((Q, L), np.float32)
    pads[1, L // 2:] = 1.0
    return ids, pads


def g8_lvt_large_t16():
    cfg = dict(models.CONFIGS[G8["cfg"]])
    cfg["vocabulary_size"] = G8["vocabulary_size"]
    var = params.synthetic_params(cfg, seed=G8["param_seed"], specs=params.clip_leaf_specs(cfg))
    x = full_video(G8["video_seed"])
    ids, pads = g8_text(G8["text_seed"], G8["Q"], G8["L"], cfg["vocabulary_size"])
    arrays = {k: np.array(v) for k, v in G8.items()}
    arrays.update(text_token_ids=ids, text_paddings=pads)
    for mode in ("f64", "bf16"):
        v, t, out = orc.video_clip(var["params"], cfg, x, ids, pads, mode,
                                   return_intermediate=("frame_embeddings",))
        arrays[f"video_emb_{mode}"] = np.asarray(v, np.float64)
        arrays[f"text_emb_{mode}"] = np.asarray(t, np.float64)
        arrays[f"similarity_{mode}"] = np.asarray(v, np.float64) @ np.asarray(t, np.float64).T
        arrays[f"frame_emb_{mode}"] = np.asarray(out["frame_embeddings"], np.float32)
    np.savez_compressed(os.path.join(HERE, "g8_lvt_large_t16.npz"), **arrays)


# LvT-Base at T = 40 (SURVEY §8(f) f1 + f3): the full-depth FactorizedVideoCLIP whose auxiliary
# encoder attends over T*N = 10240 tokens per clip (encoders.py:846-857); fp64 video / text
# embeddings, similarity and frame embeddings.
G12 = dict(cfg="videoprism_lvt_v1_base", vocabulary_size=32000, param_seed=12, video_seed=32, text_seed=42,
           Q=2, L=64, T=40)


def g12_lvt_base_t40():
    cfg = dict(models.CONFIGS[G12["cfg"]])
    cfg["vocabulary_size"] = G12["vocabulary_size"]
    var = params.synthetic_params(cfg, seed=G12["param_seed"], specs=params.clip_leaf_specs(cfg))
    x = full_video(G12["video_seed"], G12["T"])
    ids, pads = g8_text(G12["text_seed"], G12["Q"], G12["L"], cfg["vocabulary_size"])
    arrays = {k: np.array(v) for k, v in G12.items()}
    arrays.update(text_token_ids=ids, text_paddings=pads)
    v, t, out = orc.video_clip(var["params"], cfg, x, ids, pads, "f64", return_intermediate=("frame_embeddings",))
    arrays["video_emb_f64"] = np.asarray(v, np.float64)
    arrays["text_emb_f64"] = np.asarray(t, np.float64)
    arrays["similarity_f64"] = np.asarray(v, np.float64) @ np.asarray(t, np.float64).T
    arrays["frame_emb_f64"] = np.asarray(out["frame_embeddings"], np.float64)
    np.savez_compressed(os.path.join(HERE, "g12_lvt_base_t40.npz"), **arrays)


# g13: full-depth LvT-Base video embeddings of 8 clips (the construction of
# tests/test_gpu_clip.py::test_clip_full_lvt_base_bf16 at seeds 11..18: synthetic parameters and frames of the
# seed, B = 1, T = 8) in fp64, and the cast floor of each (fp64 arithmetic on bf16-rounded parameters and frames,
# mode 'wbf16'): the multi-clip bf16 gate of test_clip_lvt_base_bf16_over_clips.  ~40 s of oracle per clip.
G13_SEEDS = list(range(11, 19))


def bf16_round(a):
    u = np.ascontiguousarray(a, np.float32).view(np.uint32)
    return ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32).view(np.float32)


def g13_lvt_base_clips():
    cfg = dict(models.CONFIGS["videoprism_lvt_v1_base"])
    cfg["vocabulary_size"] = 1000
    f64, cast = [], []
    for seed in G13_SEEDS:
        var = params.synthetic_params(cfg, seed, specs=params.clip_leaf_specs(cfg))
        x = np.random.default_rng(seed).random((1, 8, 288, 288, 3), dtype=np.float32)
        f64.append(orc.video_clip(var["params"], cfg, x, None, None, "f64")[0][0])
        cast.append(orc.video_clip(var["params"], cfg, bf16_round(x), None, None, "wbf16")[0][0])
    np.savez_compressed(os.path.join(HERE, "g13_lvt_base_clips.npz"), seeds=np.array(G13_SEEDS),
                        vocabulary_size=np.array(1000), T=np.array(8), video_emb_f64=np.stack(f64),
                        cast_floor_emb=np.stack(cast))


# g14: full-depth LvT-Base at frame sizes whose token counts are not multiples of 256 (the reference's
# FactorizedVideoCLIP runs at any H = W divisible by the patch: encoders.py:505-512 interpolates the spatial
# table, :846-857 runs the auxiliary encoder over all T*N tokens, :859-885 pools any token count):
# 252 x 252 (14 x 14 = 196 patches) at T = 16 (3136 auxiliary tokens) and 144 x 144 (8 x 8) at T = 3 (192),
# B = 3 clips each, two 64-token texts.  fp64 video / text / frame embeddings and similarity, and the bf16
# cast floor of each clip's video embedding (mode 'wbf16' on bf16-rounded frames, as g13).  ~4 min of oracle.
G14 = dict(cfg="videoprism_lvt_v1_base", vocabulary_size=1000, param_seed=14, text_seed=44, Q=2, L=64, B=3)
G14_GEOM = {"s252_t16": (252, 16, 34), "s144_t3": (144, 3, 35)}


def g14_video(size, T, seed, B=3):
    return np.random.default_rng(seed).random((B, T, size, size, 3), dtype=np.float32)


def g14_lvt_base_frame_sizes():
    cfg = dict(models.CONFIGS[G14["cfg"]])
    cfg["vocabulary_size"] = G14["vocabulary_size"]
    var = params.synthetic_params(cfg, seed=G14["param_seed"], specs=params.clip_leaf_specs(cfg))
    ids, pads = g8_text(G14["text_seed"], G14["Q"], G14["L"], cfg["vocabulary_size"])
    arrays = {k: np.array(v) for k, v in G14.items()}
    arrays.update(text_token_ids=ids, text_paddings=pads)
    for tag, (size, T, vseed) in G14_GEOM.items():
        x = g14_video(size, T, vseed, G14["B"])
        v, t, out = orc.video_clip(var["params"], cfg, x, ids, pads, "f64", return_intermediate=("frame_embeddings",))
        arrays[f"{tag}/geometry"] = np.array([size, T, vseed])
        arrays[f"{tag}/video_emb_f64"] = np.asarray(v, np.float64)
        arrays[f"{tag}/text_emb_f64"] = np.asarray(t, np.float64)
        arrays[f"{tag}/similarity_f64"] = np.asarray(v, np.float64) @ np.asarray(t, np.float64).T
        arrays[f"{tag}/frame_emb_f64"] = np.asarray(out["frame_embeddings"], np.float64)
        arrays[f"{tag}/cast_floor_emb"] = np.asarray(
            orc.video_clip(var["params"], cfg, bf16_round(x), None, None, "wbf16")[0], np.float64)
        print(tag, flush=True)
    np.savez_compressed(os.path.join(HERE, "g14_lvt_base_frame_sizes.npz"), **arrays)


if __name__ == "__main__":
    which = sys.argv[1:] or ["g1", "g2", "g4", "g5", "g6", "g7", "g8", "g9", "g10", "g11", "g12", "g13", "g14"]
    if "g1" in which:
        g1_tiny()
    if "g2" in which:
        g2_base_dims()
    if "g4" in which:
        g4_ops()
    if "g5" in which:
        g5_clip_tiny()
    for tag in FULL:
        if tag.split("_")[0] in which:
            if tag in LONG:
                g_full(tag, T=LONG[tag][3], modes=("f64",))
            else:
                g_full(tag)
    if "g8" in which:
        g8_lvt_large_t16()
    if "g12" in which:
        g12_lvt_base_t40()
    if "g13" in which:
        g13_lvt_base_clips()
    if "g14" in which:
        g14_lvt_base_frame_sizes()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
