"""CPU tests of the NumPy oracle: structural pins from the reference's own tests, the
reference's own patchify call (einops, encoders.py:95-103), the committed golden fixtures,
and an independent torch-CPU restatement.  Parity against JAX itself is unpinned (JAX is
absent)."""

import os

import einops
import numpy as np
import pytest

from oracle import videoprism_oracle as orc
from videoprism import models, params
import torch_restatement

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TINY = dict(patch_size=4, pos_emb_shape=(16, 16, 16), model_dim=8, num_spatial_layers=2,
            num_temporal_layers=2, num_heads=2, mlp_dim=4, atten_logit_cap=50.0)


# ---------------- structural pins (reference tests) ----------------
def test_tiny_leaf_counts():
    """encoders_test.py:170 — 40 leaves scanned / 72 unrolled."""
    assert len(params.encoder_leaf_specs(TINY, scan=True)) == 40
    assert len(params.encoder_leaf_specs(TINY, scan=False)) == 72


@pytest.mark.parametrize("name,count", [("videoprism_v1_base", 114_365_184),
                                        ("videoprism_v1_large", 353_965_056)])
def test_param_counts(name, count):
    """README.md:34-35 (114M / 354M), recomputed exactly in SURVEY.md §0."""
    assert params.count_params(params.encoder_leaf_specs(models.CONFIGS[name])) == count


@pytest.mark.parametrize("ri,fp", [(False, False), (True, False), (False, True)])
def test_tiny_shapes(ri, fp):
    """encoders_test.py:123-181: output (1, 4*16, 8), spatial_features, frame_paddings."""
    var = params.synthetic_params(TINY, 0)
    x = np.random.default_rng(0).normal(0, 0.1, (1, 4, 16, 16, 3)).astype(np.float32)
    pads = None
    if fp:
        pads = np.zeros((1, 4), np.float32)
        pads[:, 2:] = 1
    emb, out = orc.factorized_encoder(var["params"], x, TINY, "f64", frame_paddings=pads,
                                      return_intermediate=ri)
    assert emb.shape == (1, 64, 8)
    if ri:
        assert out["spatial_features"].shape == (1, 64, 8)
    else:
        assert out == {}


# ---------------- per-op checks ----------------
def test_image_to_patch_matches_reference_einops_call():
    """The reference's exact rearrange pattern (encoders.py:95-103)."""
    x = np.random.default_rng(1).random((2, 3, 36, 54, 3))
    got = orc.image_to_patch(x, 18)
    ref = einops.rearrange(x, "... (m p)(n q) c->...(m n)(p q c)", m=2, n=3, p=18, q=18, c=3)
    np.testing.assert_array_equal(got, ref)


def test_image_to_patch_errors():
    with pytest.raises(ValueError, match="multiples"):
        orc.image_to_patch(np.zeros((1, 20, 18, 3)), 18)
    with pytest.raises(ValueError, match="4D"):
        orc.image_to_patch(np.zeros((18, 18, 3)), 18)


def test_gelu_exact_erf():
    import math
    x = np.linspace(-8, 8, 101)
    ref = np.array([0.5 * v * (1 + math.erf(v / math.sqrt(2))) for v in x])
    np.testing.assert_allclose(orc.gelu(x), ref, rtol=0, atol=1e-15)


def test_layer_norm_definition():
    """layers.py:208-270: biased var, eps inside rsqrt, (1+scale), bias."""
    rng = np.random.default_rng(2)
    x, s, b = rng.normal(size=(4, 16)), rng.normal(size=16), rng.normal(size=16)
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    ref = (x - mu) / np.sqrt(var + 1e-6) * (1 + s) + b
    np.testing.assert_allclose(orc.layer_norm(x, s, b, orc.Numerics("f64")), ref, atol=1e-12)


def test_resize_upsample_matches_mlx_restatement():
    """Upsampling = half-pixel linear + edge clamp (encoders_mlx.py:104-137)."""
    emb = np.random.default_rng(3).normal(size=(8, 5))
    ours = orc.interpolate_emb_1d(emb[None], 16)[0]
    coords = (np.arange(16) + 0.5) * (8 / 16) - 0.5
    lo = np.floor(coords)
    wu = np.clip(coords - lo, 0, 1)
    li = np.clip(lo.astype(int), 0, 7)
    ui = np.clip(lo.astype(int) + 1, 0, 7)
    ref = emb[li] * (1 - wu)[:, None] + emb[ui] * wu[:, None]
    np.testing.assert_allclose(ours, ref, atol=1e-12)


def test_resize_downsample_is_antialiased_average():
    w = orc._resize_weights(16, 4)
    np.testing.assert_allclose(w.sum(0), 1.0)
    assert np.count_nonzero(w[:, 0]) > 2          # wider than a 2-tap linear kernel
    np.testing.assert_allclose(orc._resize_weights(8, 8), np.eye(8), atol=1e-12)


def test_interpolate_2d_identity_and_errors():
    emb = np.random.default_rng(4).normal(size=(1, 16, 3))
    np.testing.assert_allclose(orc.interpolate_emb_2d(emb, (4, 4), (4, 4)), emb, atol=1e-12)
    with pytest.raises(ValueError):
        orc.interpolate_emb_2d(emb, (3, 3), (4, 4))


def test_capped_attention_uniform_when_all_masked():
    rng = np.random.default_rng(5)
    q, k, v = rng.normal(size=(3, 1, 6, 4))
    out = orc.capped_softmax_attention(q, k, v, 50.0, np.ones((1, 6)))
    np.testing.assert_allclose(out[0], np.broadcast_to(v[0].mean(0), (6, 4)), atol=1e-12)


def test_round_bf16():
    x = np.array([1.0, 1.0 + 2 ** -8, 1.0 + 3 * 2 ** -9, -2.5, 3.14159], np.float32)
    r = orc.round_bf16(x)
    assert r[0] == 1.0 and r[1] == 1.0 and r[2] == 1.0 + 2 ** -7 and r[3] == -2.5
    assert abs(r[4] - 3.140625) < 1e-7


# ---------------- golden fixtures (pin the oracle against drift) ----------------
def test_golden_tiny():
    g = np.load(os.path.join(GOLD, "g1_tiny.npz"))
    flat = {k[len("param/"):]: g[k] for k in g.files if k.startswith("param/")}
    tree = params.unflatten(flat)
    emb, out = orc.factorized_encoder(tree, g["inputs"], TINY, "f64", return_intermediate=True)
    np.testing.assert_allclose(emb, g["embeddings"], atol=1e-12)
    np.testing.assert_allclose(out["spatial_features"], g["spatial_features"], atol=1e-12)
    emb_p, _ = orc.factorized_encoder(tree, g["inputs"], TINY, "f64", frame_paddings=g["frame_paddings"])
    np.testing.assert_allclose(emb_p, g["embeddings_padded"], atol=1e-12)


def test_golden_ops():
    g = np.load(os.path.join(GOLD, "g4_ops.npz"))
    nm = orc.Numerics("f64")
    np.testing.assert_allclose(orc.layer_norm(g["ln_x"], g["ln_scale"], g["ln_bias"], nm), g["ln_out"], atol=1e-12)
    np.testing.assert_allclose(orc.gelu(g["gelu_x"]), g["gelu_y"], atol=1e-15)
    np.testing.assert_allclose(orc.capped_softmax_attention(g["att_q"], g["att_k"], g["att_v"], 50.0,
                                                            g["att_key_pad"]), g["att_out"], atol=1e-12)
    np.testing.assert_array_equal(orc.image_to_patch(g["patch_img"], 3), g["patch_out"])
    np.testing.assert_allclose(orc._resize_weights(8, 16), g["resize_up_8_16"], atol=1e-15)
    np.testing.assert_allclose(orc._resize_weights(16, 4), g["resize_down_16_4"], atol=1e-15)


@pytest.mark.slow
def test_golden_base_dims():
    g = np.load(os.path.join(GOLD, "g2_base_dims.npz"))
    cfg = dict(models.CONFIGS["videoprism_v1_base"])
    cfg.update(num_spatial_layers=2, num_temporal_layers=1)
    var = params.synthetic_params(cfg, seed=int(g["param_seed"]))
    flat = params.flatten(var["params"])
    names = sorted(flat)
    assert list(g["param_names"]) == names
    np.testing.assert_array_equal(np.stack([flat[k].ravel()[:4] for k in names]), g["param_heads"])
    x = np.random.default_rng(int(g["input_seed"])).random((1, 2, 288, 288, 3), dtype=np.float32)
    emb, _ = orc.factorized_encoder(var["params"], x, cfg, "f64")
    np.testing.assert_allclose(emb.ravel()[g["sample_index"]], g["sample_values"], atol=1e-10)
    np.testing.assert_allclose(emb.sum(-1).ravel(), g["row_sums"], atol=1e-8)


# ---------------- independent torch restatement ----------------
@pytest.mark.parametrize("padded", [False, True])
def test_oracle_vs_torch_restatement_tiny(padded):
    var = params.synthetic_params(TINY, 3)
    x = np.random.default_rng(3).normal(0, 0.1, (2, 4, 16, 16, 3)).astype(np.float32)
    fp = None
    if padded:
        fp = np.zeros((2, 4), np.float32)
        fp[0, 2:] = 1
        fp[1, :] = 1
    emb, out = orc.factorized_encoder(var["params"], x, TINY, "f64", frame_paddings=fp,
                                      return_intermediate=True)
    t_emb, t_sp = torch_restatement.factorized_encoder(var["params"], x, TINY, fp)
    np.testing.assert_allclose(emb, t_emb, atol=1e-10)
    np.testing.assert_allclose(out["spatial_features"], t_sp, atol=1e-10)


def test_oracle_vs_torch_restatement_interp():
    """pos_emb T=8 with 16 input frames (the Large interpolation path), small dims."""
    cfg = dict(TINY, pos_emb_shape=(8, 4, 4), model_dim=16, num_heads=4, mlp_dim=32)
    var = params.synthetic_params(cfg, 5)
    x = np.random.default_rng(5).random((1, 16, 16, 16, 3)).astype(np.float32)
    emb, _ = orc.factorized_encoder(var["params"], x, cfg, "f64")
    t_emb, _ = torch_restatement.factorized_encoder(var["params"], x, cfg)
    np.testing.assert_allclose(emb, t_emb, atol=1e-10)


def test_oracle_f32_and_bf16_modes_close_to_f64():
    var = params.synthetic_params(TINY, 6)
    x = np.random.default_rng(6).random((1, 4, 16, 16, 3)).astype(np.float32)
    e64, _ = orc.factorized_encoder(var["params"], x, TINY, "f64")
    e32, _ = orc.factorized_encoder(var["params"], x, TINY, "f32")
    ebf, _ = orc.factorized_encoder(var["params"], x, TINY, "bf16")
    assert np.abs(e32 - e64).max() < 1e-5
    assert 1e-4 < np.abs(ebf - e64).max() < 0.2


@pytest.mark.parametrize("mode", ["f64", "bf16"])
def test_dot_atten_query_blocks_equal_whole(monkeypatch, mode):
    """Long sequences run the oracle's attention in query blocks (the LvT auxiliary encoder over
    T*N = 10240 tokens would need 10 GB of fp64 logits at once); each query row's softmax is
    independent of the others, so the blocked form equals the whole one, with key paddings too."""
    rng = np.random.default_rng(11)
    B, S, N, H = 2, 37, 3, 8
    q, k, v = (rng.normal(0, 1.0, (B, S, N, H)) for _ in range(3))
    pad = np.zeros((B, S))
    pad[1, 30:] = 1.0
    nm = orc.Numerics(mode)
    for mask in (None, orc.padding_mask(pad), orc.attention_masks_for_fprop(pad, True)):
        whole = orc.dot_atten(q, k, v, mask, nm, 50.0, H)
        monkeypatch.setattr(orc, "_ATTN_CHUNK_ELEMS", B * N * S * 5)  # 5 query rows per block
        blocked = orc.dot_atten(q, k, v, mask, nm, 50.0, H)
        monkeypatch.undo()
        np.testing.assert_allclose(blocked, whole, rtol=0, atol=1e-14 if mode == "f64" else 0)


def test_golden_lvt_base_clips_fixture():
    """g13 (the multi-clip LvT-Base bf16 gate): L2-normalised fp64 embeddings of 8 clips, and cast floors
    that are the bf16 noise the gate measures against -- non-zero and of the order of the 1e-3 bar."""
    g = np.load(os.path.join(GOLD, "g13_lvt_base_clips.npz"))
    assert list(g["seeds"]) == list(range(11, 19))
    e, c = g["video_emb_f64"], g["cast_floor_emb"]
    assert e.shape == c.shape == (8, 768)
    np.testing.assert_allclose(np.linalg.norm(e, axis=-1), 1.0, rtol=1e-12)
    floor = np.abs(c - e).max(axis=-1)
    assert bool(((floor > 5e-4) & (floor < 2e-3)).all()), floor
