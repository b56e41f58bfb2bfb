"""Drop-in for videoprism/models_mlx.py (models_mlx.py:14-316) on MI355X.

`load_video_encoder(name, weights_path)` returns a callable encoder:
`model(video, return_intermediate=False, frame_paddings=None) -> (emb, outputs)`
(encoders_mlx.py:502-543).  Weights: the files the reference's convert_weights.py
writes (`weights/{name}_mlx.safetensors` or `.npz`, unstacked `layers/{i}` keys) or
a Flax "repeated" npz; both are converted to the canonical scanned layout.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np

from . import encoders
from . import params as params_lib
from . import utils

MODEL_CONFIGS = {
    "videoprism_public_v1_base": {
        "patch_size": 18, "pos_emb_shape": (16, 16, 16), "model_dim": 768,
        "num_spatial_layers": 12, "num_temporal_layers": 4, "num_heads": 12, "mlp_dim": 3072,
        "atten_logit_cap": 50.0, "norm_policy": "pre"},
    "videoprism_public_v1_large": {
        "patch_size": 18, "pos_emb_shape": (8, 16, 16), "model_dim": 1024,
        "num_spatial_layers": 24, "num_temporal_layers": 4, "num_heads": 16, "mlp_dim": 4096,
        "atten_logit_cap": 50.0, "norm_policy": "pre"},
    "videoprism_lvt_public_v1_base": {
        "patch_size": 18, "pos_emb_shape": (16, 16, 16), "num_spatial_layers": 12,
        "num_temporal_layers": 4, "mlp_dim": 3072, "num_auxiliary_layers": 2,
        "vocabulary_size": 32000, "enable_causal_atten": True, "num_unimodal_layers": 12,
        "norm_policy": "pre", "model_dim": 768, "num_heads": 12, "atten_logit_cap": 50.0},
    "videoprism_lvt_public_v1_large": {
        "patch_size": 18, "pos_emb_shape": (8, 16, 16), "num_spatial_layers": 24,
        "num_temporal_layers": 4, "mlp_dim": 4096, "num_auxiliary_layers": 2,
        "vocabulary_size": 32000, "enable_causal_atten": True, "num_unimodal_layers": 12,
        "norm_policy": "pre", "model_dim": 1024, "num_heads": 16, "atten_logit_cap": 50.0},
}


def get_model_config(model_name: str) -> dict:
    """models_mlx.py:72-88."""
    if model_name not in MODEL_CONFIGS:
        available = ", ".join(MODEL_CONFIGS.keys())
        raise ValueError(f"Model '{model_name}' not found. Available models: {available}")
    return MODEL_CONFIGS[model_name].copy()


def _resolve(model_name: str, weights_path) -> Path:
    if weights_path is None:
        weights_dir = Path("weights")
        weights_path = weights_dir / f"{model_name}_mlx.safetensors"
        if not weights_path.exists():
            weights_path = weights_dir / f"{model_name}_mlx.npz"
    else:
        weights_path = Path(weights_path)
    if not weights_path.exists():
        raise FileNotFoundError(f"Weights not found at {weights_path}. "
                                f"Please run: python convert_weights.py")
    return weights_path


def load_weights_from_file(filepath: str) -> dict:
    """models_mlx.py:297-316 — flat {name: array}."""
    filepath = Path(filepath)
    if not filepath.exists():
        raise FileNotFoundError(f"File not found: {filepath}")
    if filepath.suffix == ".safetensors":
        from safetensors.numpy import load_file
        return dict(load_file(str(filepath)))
    if filepath.suffix == ".npz":
        return dict(np.load(str(filepath), allow_pickle=False))
    raise ValueError(f"Unsupported file format: {filepath.suffix}")


class VideoEncoder:
    """Callable wrapper: `model(video, return_intermediate=False, frame_paddings=None)`."""

    def __init__(self, config: dict, variables: dict, fprop_dtype=None):
        cfg = {k: v for k, v in config.items() if k != "norm_policy"}
        self.encoder = encoders.FactorizedEncoder(norm_policy=config.get("norm_policy", "pre"),
                                                  fprop_dtype=fprop_dtype, **cfg)
        self.variables = variables

    def __call__(self, inputs, return_intermediate=False, frame_paddings=None):
        return self.encoder.apply(self.variables, inputs, train=False,
                                  return_intermediate=return_intermediate,
                                  frame_paddings=frame_paddings)


def load_video_encoder(model_name: str, weights_path: str = None, fprop_dtype=None) -> VideoEncoder:
    """models_mlx.py:146-210."""
    config = get_model_config(model_name)
    if "lvt" in model_name:
        raise ValueError(
            f"Model '{model_name}' is a video-text model. Use load_model() instead, or use a "
            f"video-only model like 'videoprism_public_v1_base' or 'videoprism_public_v1_large'")
    path = _resolve(model_name, weights_path)
    flat = load_weights_from_file(str(path))
    canonical = params_lib.canonical_params(flat)
    # drop an 'params/' or 'vision_encoder/' prefix if the file carries one
    canonical = {k.split("vision_encoder/", 1)[-1]: v for k, v in canonical.items()}
    return VideoEncoder(config, {"params": utils.recover_tree(list(canonical), list(canonical.values()))},
                        fprop_dtype=fprop_dtype)


class VideoCLIP:
    """Callable wrapper of the LvT model (encoders_mlx.py:826-910 call signature):
    `model(inputs=None, text_token_ids=None, text_paddings=None, normalize=True,
    return_intermediate=False, frame_paddings=None) -> (video_emb, text_emb, outputs)`."""

    def __init__(self, config: dict, variables: dict, fprop_dtype=None):
        cfg = {k: v for k, v in config.items()}
        self.model = encoders.FactorizedVideoCLIP(fprop_dtype=fprop_dtype, **cfg)
        self.variables = variables

    def __call__(self, inputs=None, text_token_ids=None, text_paddings=None, normalize=True,
                 return_intermediate=False, frame_paddings=None):
        return self.model.apply(self.variables, inputs, text_token_ids, text_paddings,
                                train=False, normalize=normalize,
                                return_intermediate=return_intermediate,
                                frame_paddings=frame_paddings)


def load_model(model_name: str, weights_path: str = None, fprop_dtype=None) -> VideoCLIP:
    """models_mlx.py:91-143: the LvT video-text model from a local weights file (a Flax
    "repeated" npz of the full model, or unstacked `layers/{i}` keys)."""
    config = get_model_config(model_name)
    path = _resolve(model_name, weights_path)
    flat = load_weights_from_file(str(path))
    canonical = params_lib.canonical_params(flat)
    return VideoCLIP(config, {"params": utils.recover_tree(list(canonical), list(canonical.values()))},
                     fprop_dtype=fprop_dtype)


def load_classifier(model_name: str, num_classes: int, weights_path: str = None, fprop_dtype=None):
    """models_mlx.py:213-294: a FactorizedVideoClassifier on the named model's encoder (for LvT
    names the vision encoder's hyper-parameters).  Pre-trained files hold the encoder only, so the
    pooler and the projection start from the Flax initialisers' distributions (deterministic numpy
    draws) -- the reference likewise loads only the encoder weights; returns (model, variables)."""
    config = get_model_config(model_name)
    enc = {k: config[k] for k in ("patch_size", "pos_emb_shape", "model_dim", "num_spatial_layers",
                                  "num_temporal_layers", "num_heads", "mlp_dim", "atten_logit_cap")}
    model = encoders.FactorizedVideoClassifier(encoder_params=enc, num_classes=num_classes,
                                               fprop_dtype=fprop_dtype)
    variables = model.init(0)
    if weights_path is not None:
        flat = load_weights_from_file(str(_resolve(model_name, weights_path)))
        canonical = params_lib.canonical_params(flat)
        tree = params_lib.flatten(variables["params"])
        for k, v in canonical.items():
            k = k[len("vision_encoder/"):] if k.startswith("vision_encoder/") else k
            k = k[len("encoder/"):] if k.startswith("encoder/") else k
            key = "encoder/" + k
            if key in tree:
                tree[key] = v
        variables = {"params": params_lib.unflatten(tree)}
    return model, variables
