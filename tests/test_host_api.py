"""Host-side drop-in API (models / models_mlx / utils / params), mirroring the reference's
models_test.py and error behaviour.  No GPU: nothing here reaches a kernel."""

import numpy as np
import pytest

from videoprism import encoders, models, models_mlx, params, utils

TINY = dict(patch_size=4, pos_emb_shape=(16, 16, 16), model_dim=8, num_spatial_layers=2,
            num_temporal_layers=2, num_heads=2, mlp_dim=4, atten_logit_cap=50.0)


@pytest.mark.parametrize("name,exists", [("videoprism_public_v1_base", True),
                                         ("videoprism_public_v1_large", True),
                                         ("videoprism_public_v1_giant", False),
                                         ("google/videoprism-base-f16r288", True),
                                         ("google/nope", False)])
def test_has_model(name, exists):
    """models_test.py:28-34."""
    assert models.has_model(name) == exists


def test_get_model_and_errors():
    m = models.get_model("videoprism_public_v1_base")
    assert isinstance(m, encoders.FactorizedEncoder)
    assert (m.model_dim, m.num_spatial_layers, m.atten_logit_cap) == (768, 12, 50.0)
    assert not m.is_bf16
    import torch
    mb = models.get_model("google/videoprism-large-f8r288", fprop_dtype=torch.bfloat16)
    assert mb.is_bf16 and mb.model_dim == 1024 and tuple(mb.pos_emb_shape) == (8, 16, 16)
    with pytest.raises(ValueError, match="not found"):
        models.get_model("videoprism_public_v1_giant")
    lvt = models.get_model("videoprism_lvt_public_v1_base")
    assert isinstance(lvt, encoders.FactorizedVideoCLIP)
    assert (lvt.model_dim, lvt.num_auxiliary_layers, lvt.vocabulary_size) == (768, 2, 32000)
    with pytest.raises(ValueError, match="missing parameters"):
        lvt.engine({"params": {}}, 0)


def test_init_leaf_count_and_shapes():
    """encoders_test.py:170 — 40 leaves for the scanned tiny encoder."""
    enc = encoders.FactorizedEncoder(**TINY)
    var = enc.init(0, None)
    flat = params.flatten(var["params"])
    assert len(flat) == 40
    params.validate(flat, enc.param_specs())
    assert np.all(flat["spatial_ln/scale"] == 0)  # LayerNorm scale init 0 (layers.py:248)


def test_load_pretrained_weights_local_roundtrip(tmp_path):
    var = params.synthetic_params(TINY, 1)
    path = tmp_path / "ckpt.npz"
    np.savez(path, **{"params/" + k: v for k, v in params.flatten(var["params"]).items()})
    loaded = models.load_pretrained_weights(None, checkpoint_path=str(path))
    assert set(loaded) == {"params"}
    flat = params.flatten(loaded["params"])
    for k, v in params.flatten(var["params"]).items():
        np.testing.assert_array_equal(flat[k], v)
    with pytest.raises(FileNotFoundError):
        models.load_pretrained_weights("videoprism_public_v1_base")


def test_recover_tree():
    """utils.py:84-105."""
    t = utils.recover_tree(["a/b/c", "a/d", "e"], [1, 2, 3])
    assert t == {"a": {"b": {"c": 1}, "d": 2}, "e": 3}
    with pytest.raises(ValueError):
        utils.npload("gs://bucket/x.npz")


def test_canonical_params_from_mlx_layout():
    """convert_weights.py:88-202 layout (unstacked layers/i, kernel/scale/emb_var -> weight)
    maps back to the scanned Flax layout."""
    var = params.synthetic_params(TINY, 2)
    flat = params.flatten(var["params"])
    mlx = {}
    for k, v in flat.items():
        nk = k.replace("/kernel", "/weight").replace("/scale", "/weight").replace("/emb_var", "/weight")
        if "/x_layers/" in nk:
            for i in range(v.shape[0]):
                mlx[nk.replace("/x_layers/", f"/layers/{i}/")] = v[i]
        else:
            mlx[nk] = v
    back = params.canonical_params(mlx)
    params.validate(back, params.encoder_leaf_specs(TINY))
    for k, v in flat.items():
        np.testing.assert_array_equal(back[k], v)


def test_canonical_params_unrolled_flax():
    var = params.synthetic_params(TINY, 3)
    flat = params.flatten(var["params"])
    unrolled = {}
    for k, v in flat.items():
        if "/x_layers/" in k:
            for i in range(v.shape[0]):
                unrolled[k.replace("/x_layers/", f"/x_layers_{i}/")] = v[i]
        else:
            unrolled[k] = v
    assert len(unrolled) == 72  # encoders_test.py:170 unrolled count
    back = params.canonical_params({"params": params.unflatten(unrolled)})
    for k, v in flat.items():
        np.testing.assert_array_equal(back[k], v)


def test_validate_errors():
    specs = params.encoder_leaf_specs(TINY)
    flat = params.flatten(params.synthetic_params(TINY, 0)["params"])
    bad = dict(flat)
    del bad["temporal_ln/bias"]
    with pytest.raises(ValueError, match="missing"):
        params.validate(bad, specs)
    bad = dict(flat)
    bad["spatial_ln/bias"] = np.zeros(3, np.float32)
    with pytest.raises(ValueError, match="shape mismatch"):
        params.validate(bad, specs)


def test_models_mlx_surface(tmp_path):
    """models_mlx.py:72-88, :146-210 error behaviour."""
    with pytest.raises(ValueError, match="not found"):
        models_mlx.get_model_config("nope")
    cfg = models_mlx.get_model_config("videoprism_public_v1_base")
    assert cfg["model_dim"] == 768 and cfg["norm_policy"] == "pre"
    with pytest.raises(ValueError, match="video-text"):
        models_mlx.load_video_encoder("videoprism_lvt_public_v1_base")
    with pytest.raises(FileNotFoundError):
        models_mlx.load_video_encoder("videoprism_public_v1_base", weights_path=str(tmp_path / "x.npz"))
    with pytest.raises(ValueError, match="Unsupported"):
        p = tmp_path / "w.bin"
        p.write_bytes(b"")
        models_mlx.load_weights_from_file(str(p))


def test_models_mlx_loads_converted_file(tmp_path):
    """A file in convert_weights.py's layout builds an encoder whose params validate."""
    cfg = models_mlx.get_model_config("videoprism_public_v1_base")
    var = params.synthetic_params(models.CONFIGS["videoprism_v1_base"], 0)
    flat = params.flatten(var["params"])
    mlx = {}
    for k, v in flat.items():
        nk = k.replace("/kernel", "/weight").replace("/scale", "/weight").replace("/emb_var", "/weight")
        if "/x_layers/" in nk:
            for i in range(v.shape[0]):
                mlx[nk.replace("/x_layers/", f"/layers/{i}/")] = v[i]
        else:
            mlx[nk] = v
    path = tmp_path / "videoprism_public_v1_base_mlx.npz"
    np.savez(path, **mlx)
    enc = models_mlx.load_video_encoder("videoprism_public_v1_base", weights_path=str(path))
    back = params.canonical_params(enc.variables)
    params.validate(back, enc.encoder.param_specs())
    assert enc.encoder.model_dim == cfg["model_dim"]
