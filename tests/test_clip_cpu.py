"""CPU tests of the LvT video-text path: structural pins from the
reference's own FactorizedVideoCLIP test (encoders_test.py:283-360), the oracle against the
independent torch restatement and the committed golden fixture, and the host-side API.
Value parity against JAX itself is unpinned (JAX absent)."""

import os

import numpy as np
import pytest

from oracle import videoprism_oracle as orc
from videoprism import encoders, models, models_mlx, params
import torch_restatement

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# encoders_test.py:308-324
CLIP_TINY = dict(patch_size=4, pos_emb_shape=(16, 16, 16), num_spatial_layers=2, num_temporal_layers=2,
                 mlp_dim=4, num_auxiliary_layers=1, vocabulary_size=20, enable_causal_atten=True,
                 num_unimodal_layers=2, model_dim=8, num_heads=2, atten_logit_cap=50.0)


def _inputs(seed=0):
    rng = np.random.default_rng(seed)
    x = rng.normal(0.0, 0.1, (1, 4, 16, 16, 3)).astype(np.float32)
    ids = rng.integers(0, 20, (1, 10)).astype(np.int32)
    pads = np.zeros((1, 10), np.float32)
    pads[:, 5:] = 1.0
    return x, ids, pads


def test_clip_leaf_counts():
    """encoders_test.py:339 — 88 leaves scanned, 136 unrolled."""
    assert len(params.clip_leaf_specs(CLIP_TINY, scan=True)) == 88
    assert len(params.clip_leaf_specs(CLIP_TINY, scan=False)) == 136


def test_pooler_leaf_count():
    """layers_test.py:283 — AttenTokenPoolingLayer has 12 leaves."""
    specs = params.clip_leaf_specs(CLIP_TINY)
    assert len([k for k in specs if k.startswith("contrastive_vision_pooler/")]) == 12


@pytest.mark.parametrize("ri", [False, True, ("spatial_features",), ("frame_embeddings",)])
def test_clip_tiny_shapes(ri):
    """encoders_test.py:340-360: embeddings (1, 8); intermediate keys as requested."""
    var = params.synthetic_params(CLIP_TINY, 0, specs=params.clip_leaf_specs(CLIP_TINY))
    x, ids, pads = _inputs()
    v, t, out = orc.video_clip(var["params"], CLIP_TINY, x, ids, pads, return_intermediate=ri)
    assert v.shape == (1, 8) and t.shape == (1, 8)
    np.testing.assert_allclose(np.linalg.norm(v, axis=-1), 1.0, rtol=1e-12)
    np.testing.assert_allclose(np.linalg.norm(t, axis=-1), 1.0, rtol=1e-12)
    if ri is False:
        assert out == {}
    elif ri is True:
        assert set(out) == {"frame_embeddings", "spatial_features", "spatiotemporal_features"}
        assert out["spatial_features"].shape == (1, 64, 8)
        assert out["frame_embeddings"].shape == (1, 4, 8)
    else:
        assert set(out) == set(ri)


def test_clip_video_or_text_only():
    var = params.synthetic_params(CLIP_TINY, 0, specs=params.clip_leaf_specs(CLIP_TINY))
    x, ids, pads = _inputs()
    v, t, _ = orc.video_clip(var["params"], CLIP_TINY, inputs=x)
    assert t is None and v.shape == (1, 8)
    v, t, _ = orc.video_clip(var["params"], CLIP_TINY, text_token_ids=ids, text_paddings=pads)
    assert v is None and t.shape == (1, 8)
    with pytest.raises(AssertionError, match="Text paddings"):
        orc.video_clip(var["params"], CLIP_TINY, text_token_ids=ids)


@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_clip_vs_torch_restatement(seed):
    var = params.synthetic_params(CLIP_TINY, seed, specs=params.clip_leaf_specs(CLIP_TINY))
    x, ids, pads = _inputs(seed)
    v, t, out = orc.video_clip(var["params"], CLIP_TINY, x, ids, pads, return_intermediate=True)
    v2, t2, f2 = torch_restatement.video_clip(var["params"], CLIP_TINY, x, ids, pads)
    np.testing.assert_allclose(v, v2, atol=1e-12)
    np.testing.assert_allclose(t, t2, atol=1e-12)
    np.testing.assert_allclose(out["frame_embeddings"], f2, atol=1e-12)


def test_golden_clip_tiny():
    g = np.load(os.path.join(GOLD, "g5_clip_tiny.npz"), allow_pickle=False)
    flat = {k[len("param/"):]: g[k] for k in g.files if k.startswith("param/")}
    tree = params.unflatten(flat)
    v, t, out = orc.video_clip(tree, CLIP_TINY, g["inputs"], g["text_token_ids"], g["text_paddings"],
                               return_intermediate=True)
    np.testing.assert_allclose(v, g["video_embeddings"], atol=1e-13)
    np.testing.assert_allclose(t, g["text_embeddings"], atol=1e-13)
    np.testing.assert_allclose(out["frame_embeddings"], g["frame_embeddings"], atol=1e-13)


def test_causal_mask_merge_semantics():
    """layers.py:111-179: padded queries are fully masked when causal; otherwise keys only."""
    pad = np.array([[0.0, 0.0, 1.0]])
    m = orc.attention_masks_for_fprop(pad, causal=True)[0, 0] < 0
    assert m.tolist() == [[False, True, True], [False, False, True], [True, True, True]]
    m = orc.attention_masks_for_fprop(pad, causal=False)[0, 0] < 0
    assert m.tolist() == [[False, False, True]]


def test_masked_attention_uniform_rows():
    rng = np.random.default_rng(0)
    q, k, v = rng.normal(0, 1, (3, 2, 5, 4))
    pad = np.array([[0, 0, 0, 1, 1], [1, 0, 0, 0, 0]], np.float64)
    out = orc.masked_attention(q, k, v, 50.0, pad, causal=True)
    # padded query rows (row 3, 4 of seq 0; row 0 of seq 1) average every value row
    np.testing.assert_allclose(out[0, 3], v[0].mean(0), atol=1e-12)
    np.testing.assert_allclose(out[1, 0], v[1].mean(0), atol=1e-12)
    # query 0 of seq 0 sees only key 0
    np.testing.assert_allclose(out[0, 0], v[0, 0], atol=1e-12)


def test_sinusoidal_positions():
    """encoders.py:190-224: [sin | cos] with log-spaced timescales 1..1e4."""
    e = orc.sinusoidal_positions(3, 8)
    inv = np.exp(-np.arange(4) * np.log(1e4) / 3)
    np.testing.assert_allclose(e[2], np.concatenate([np.sin(2 * inv), np.cos(2 * inv)]), atol=1e-15)
    assert orc.sinusoidal_positions(2, 5).shape == (2, 5)


def test_host_clip_api_surface():
    m = models.get_model("google/videoprism-lvt-large-f8r288")
    assert isinstance(m, encoders.FactorizedVideoCLIP)
    assert (m.model_dim, m.num_heads, m.num_unimodal_layers, m.vocabulary_size) == (1024, 16, 12, 32000)
    var = m.init(0)
    assert len(params.flatten(var["params"])) == 88
    with pytest.raises(FileNotFoundError):
        models_mlx.load_model("videoprism_lvt_public_v1_base", weights_path="/nonexistent.npz")
    with pytest.raises(ValueError, match="not found"):
        models_mlx.load_model("videoprism_lvt_public_v1_giant")


# ---------------- FactorizedVideoClassifier (encoders.py:583-653) ----------------
ENC_TINY = dict(patch_size=4, pos_emb_shape=(16, 16, 16), model_dim=8, num_spatial_layers=2,
                num_temporal_layers=2, num_heads=2, mlp_dim=4, atten_logit_cap=50.0)


def test_classifier_leaf_count():
    """encoders_test.py:224 — 54 leaves."""
    assert len(params.classifier_leaf_specs(ENC_TINY, 10)) == 54


@pytest.mark.parametrize("ri", [False, True])
def test_classifier_tiny_shapes(ri):
    """encoders_test.py:205-240: logits (B, 10); intermediates spatial / spatiotemporal / global."""
    var = params.synthetic_params(ENC_TINY, 0, specs=params.classifier_leaf_specs(ENC_TINY, 10))
    x = np.random.default_rng(0).normal(0, 0.1, (2, 4, 16, 16, 3)).astype(np.float32)
    logits, out = orc.video_classifier(var["params"], ENC_TINY, x, return_intermediate=ri)
    assert logits.shape == (2, 10)
    if ri:
        assert set(out) == {"spatial_features", "spatiotemporal_features", "global_embeddings"}
        assert out["global_embeddings"].shape == (2, 8)
    else:
        assert out == {}


def test_classifier_registry_and_loader():
    m = models.videoprism_vc_v1_large(7)
    assert isinstance(m, encoders.FactorizedVideoClassifier)
    assert m.num_classes == 7 and m.encoder_params["model_dim"] == 1024
    mm, var = models_mlx.load_classifier("videoprism_lvt_public_v1_base", 3)
    assert len(params.flatten(var["params"])) == 54
    assert var["params"]["projection"]["linear"]["kernel"].shape == (768, 3)


def test_oracle_classifier_vs_torch_restatement():
    var = params.synthetic_params(ENC_TINY, 3, specs=params.classifier_leaf_specs(ENC_TINY, 10))
    x = np.random.default_rng(3).normal(0, 0.1, (2, 4, 16, 16, 3)).astype(np.float32)
    logits, _ = orc.video_classifier(var["params"], ENC_TINY, x)
    np.testing.assert_allclose(logits, torch_restatement.video_classifier(var["params"], ENC_TINY, x), atol=1e-11)


def _convert_like_reference(flat: dict, cfg: dict, lvt: bool) -> dict:
    """Restates convert_weights.py:88-104 (rename_parameter) and :107-226 (convert_flax_to_mlx):
    scanned stacks listed by component are unstacked to `<prefix>/layers/{i}/...` (only when
    dim 0 == the component's layer count), then '/kernel', '/scale', '/emb_var' -> '/weight'
    everywhere.  Test-side restatement; the reference script itself needs flax."""
    def rename(n):
        return n.replace("/kernel", "/weight").replace("/scale", "/weight").replace("/emb_var", "/weight")
    vp = "vision_encoder/" if lvt else ""
    comps = [(f"{vp}spatial_encoder/transformers_stack", cfg["num_spatial_layers"]),
             (f"{vp}temporal_encoder/transformers_stack", cfg["num_temporal_layers"])]
    if lvt:
        comps += [("text_encoder/unimodal_transformer", cfg["num_unimodal_layers"]),
                  ("auxiliary_encoder/transformers_stack", cfg["num_auxiliary_layers"])]
    out = {}
    for prefix, L in comps:
        for k, v in flat.items():
            if k.startswith(prefix) and "/x_layers/" in k:
                leaf = k.split("/x_layers/", 1)[1]
                if v.ndim > 0 and v.shape[0] == L:
                    for i in range(L):
                        out[rename(f"{prefix}/layers/{i}/{leaf}")] = v[i]
    for k, v in flat.items():
        if "/x_layers/" not in k:
            out[rename(k)] = v
    return out


def test_load_model_reference_converted_lvt(tmp_path):
    """A LvT tree renamed and unstacked by convert_weights.py's rules (incl. text_encoder/
    token_emb/emb_var -> .../weight, mapped back as weight_utils.py:33-34 does) loads through
    models_mlx.load_model with every leaf bit-identical."""
    cfg = dict(models.CONFIGS["videoprism_lvt_v1_base"])
    cfg.update(num_spatial_layers=2, num_temporal_layers=1, num_auxiliary_layers=2,
               num_unimodal_layers=3, vocabulary_size=50)
    var = params.synthetic_params(cfg, seed=4, specs=params.clip_leaf_specs(cfg))
    flat = params.flatten(var["params"])
    conv = _convert_like_reference(flat, cfg, lvt=True)
    assert "text_encoder/token_emb/weight" in conv
    assert len(conv) == sum(v.shape[0] if "/x_layers/" in k else 1 for k, v in flat.items())
    path = tmp_path / "videoprism_lvt_public_v1_base_mlx.safetensors"
    from safetensors.numpy import save_file
    save_file({k: np.ascontiguousarray(v) for k, v in conv.items()}, str(path))
    clip = models_mlx.load_model("videoprism_lvt_public_v1_base", weights_path=str(path))
    back = params.canonical_params(clip.variables)
    specs = params.clip_leaf_specs(cfg)
    params.validate(back, specs)
    for k, v in flat.items():
        np.testing.assert_array_equal(back[k], v)


def test_canonical_params_renamed_but_stacked():
    """Keys renamed to '/weight' while the stacks stay scanned still map back."""
    cfg = dict(CLIP_TINY)
    var = params.synthetic_params(cfg, seed=5, specs=params.clip_leaf_specs(cfg))
    flat = params.flatten(var["params"])
    ren = {k.replace("/kernel", "/weight").replace("/scale", "/weight").replace("/emb_var", "/weight"): v
           for k, v in flat.items()}
    back = params.canonical_params(ren)
    params.validate(back, params.clip_leaf_specs(cfg))
