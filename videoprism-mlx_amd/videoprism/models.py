"""Model registry and loaders — the drop-in for videoprism/models.py.

Same names and behaviour as the reference (models.py:54-336): `CONFIGS`, `MODELS`,
`CHECKPOINTS`, `has_model`, `get_model(model_name, model_fn, models, fprop_dtype)`,
`load_pretrained_weights(model_name, checkpoint_path, checkpoints)`.  The returned model
runs its forward on MI355X through libvideoprism_hip.so.

Differences, all forced by the offline deployment: `load_pretrained_weights` needs a
local `checkpoint_path` (or a path in `checkpoints`) instead of a Hugging Face download.
LvT (video-text) models return `encoders.FactorizedVideoCLIP` (encoders.py:762-910), whose
`apply(variables, inputs, text_token_ids, text_paddings, ...)` runs both towers on MI355X;
text tokenisation itself (tokenizers.py, sentencepiece model download) is out of scope, so
callers pass token ids.
"""

from __future__ import annotations

import functools
import os
from collections.abc import Callable, Mapping

from . import encoders
from . import utils

K400_NUM_CLASSES: int = 400
SSV2_NUM_CLASSES: int = 174
TEXT_MAX_LEN: int = 64
TEXT_TOKENIZERS = {
    "c4_en": {
        "model_path": "gs://t5-data/vocabs/cc_en.32000/sentencepiece.model",
        "vocab_size": 32_000,
    },
}

CHECKPOINTS = {
    "videoprism_public_v1_base": ("google/videoprism-base-f16r288", "flax_base_f16r288_repeated.npz"),
    "videoprism_public_v1_large": ("google/videoprism-large-f8r288", "flax_large_f8r288_repeated.npz"),
    "videoprism_lvt_public_v1_base": ("google/videoprism-lvt-base-f16r288", "flax_lvt_base_f16r288_repeated.npz"),
    "videoprism_lvt_public_v1_large": ("google/videoprism-lvt-large-f8r288", "flax_lvt_large_f8r288_repeated.npz"),
}

CONFIGS = {
    "videoprism_v1_base": dict(
        patch_size=18, pos_emb_shape=(16, 16, 16), model_dim=768, num_spatial_layers=12,
        num_temporal_layers=4, num_heads=12, mlp_dim=3072, atten_logit_cap=50.0, scan=True),
    "videoprism_v1_large": dict(
        patch_size=18, pos_emb_shape=(8, 16, 16), model_dim=1024, num_spatial_layers=24,
        num_temporal_layers=4, num_heads=16, mlp_dim=4096, atten_logit_cap=50.0, scan=True),
    "videoprism_v1_giant": dict(
        patch_size=18, pos_emb_shape=(8, 16, 16), model_dim=1408, num_spatial_layers=40,
        num_temporal_layers=4, num_heads=16, mlp_dim=6144, atten_logit_cap=50.0, scan=True),
    "videoprism_lvt_v1_base": dict(
        patch_size=18, pos_emb_shape=(16, 16, 16), num_spatial_layers=12, num_temporal_layers=4,
        mlp_dim=3072, num_auxiliary_layers=2, enable_causal_atten=True, num_unimodal_layers=12,
        norm_policy="pre", model_dim=768, num_heads=12, atten_logit_cap=50.0, scan=True),
    "videoprism_lvt_v1_large": dict(
        patch_size=18, pos_emb_shape=(8, 16, 16), num_spatial_layers=24, num_temporal_layers=4,
        mlp_dim=4096, num_auxiliary_layers=2, enable_causal_atten=True, num_unimodal_layers=12,
        norm_policy="pre", model_dim=1024, num_heads=16, atten_logit_cap=50.0, scan=True),
    "videoprism_lvt_v1_giant": dict(
        patch_size=18, pos_emb_shape=(8, 16, 16), num_spatial_layers=40, num_temporal_layers=4,
        mlp_dim=6144, num_auxiliary_layers=2, enable_causal_atten=True, num_unimodal_layers=16,
        norm_policy="primer_hybrid", model_dim=1408, num_heads=16, atten_logit_cap=50.0, scan=True),
}


def videoprism_v1_base():
    return encoders.FactorizedEncoder(**CONFIGS["videoprism_v1_base"])


def videoprism_v1_large():
    return encoders.FactorizedEncoder(**CONFIGS["videoprism_v1_large"])


def videoprism_v1_giant():
    return encoders.FactorizedEncoder(**CONFIGS["videoprism_v1_giant"])


def videoprism_lvt_v1_base(text_tokenizer: str = "c4_en"):
    config = dict(CONFIGS["videoprism_lvt_v1_base"])
    config["vocabulary_size"] = TEXT_TOKENIZERS[text_tokenizer]["vocab_size"]
    return encoders.FactorizedVideoCLIP(**config)


def videoprism_lvt_v1_large(text_tokenizer: str = "c4_en"):
    config = dict(CONFIGS["videoprism_lvt_v1_large"])
    config["vocabulary_size"] = TEXT_TOKENIZERS[text_tokenizer]["vocab_size"]
    return encoders.FactorizedVideoCLIP(**config)


def videoprism_vc_v1_base(num_classes: int):
    """models.py:195-200: FactorizedVideoClassifier on the Base encoder."""
    return encoders.FactorizedVideoClassifier(encoder_params=dict(CONFIGS["videoprism_v1_base"]),
                                              num_classes=num_classes)


def videoprism_vc_v1_large(num_classes: int):
    return encoders.FactorizedVideoClassifier(encoder_params=dict(CONFIGS["videoprism_v1_large"]),
                                              num_classes=num_classes)


def videoprism_vc_v1_giant(num_classes: int):
    return encoders.FactorizedVideoClassifier(encoder_params=dict(CONFIGS["videoprism_v1_giant"]),
                                              num_classes=num_classes)


MODELS = {
    "videoprism_public_v1_base": videoprism_v1_base,
    "videoprism_public_v1_large": videoprism_v1_large,
    "videoprism_lvt_public_v1_base": functools.partial(videoprism_lvt_v1_base, text_tokenizer="c4_en"),
    "videoprism_lvt_public_v1_large": functools.partial(videoprism_lvt_v1_large, text_tokenizer="c4_en"),
}


def _get_model_name_by_hf_model_id(model_id: str) -> str | None:
    """models.py:236-252."""
    for model_name, value in CHECKPOINTS.items():
        if isinstance(value, tuple) and value[0] == model_id:
            return model_name
    return None


def has_model(model_name: str, models: Mapping[str, Callable] | None = None) -> bool:
    """models.py:255-265."""
    models = models or MODELS
    if model_name.startswith("google/"):
        model_name = _get_model_name_by_hf_model_id(model_name)
    return model_name is not None and model_name in models


def get_model(model_name: str | None, model_fn: Callable | None = None,
              models: Mapping[str, Callable] | None = None, fprop_dtype=None):
    """models.py:268-303."""
    if model_fn is None:
        assert model_name is not None
        models = models or MODELS
        if model_name.startswith("google/"):
            model_name = _get_model_name_by_hf_model_id(model_name)
            if model_name is None:
                raise ValueError(f"Failed to find model name with `{model_name}`.")
        if model_name not in models:
            raise ValueError(f"Model `{model_name}` not found.")
        model_fn = models[model_name]
    model = model_fn()
    if fprop_dtype is not None:
        model.fprop_dtype = fprop_dtype
    return model


def load_pretrained_weights(model_name: str | None, checkpoint_path: str | None = None,
                            checkpoints: Mapping | None = None):
    """models.py:306-336 with local files only.  Returns {'params': tree} (numpy)."""
    checkpoints = checkpoints or CHECKPOINTS
    if checkpoint_path is None:
        assert model_name is not None
        if model_name.startswith("google/"):
            model_name = _get_model_name_by_hf_model_id(model_name)
        entry = checkpoints[model_name]
        if isinstance(entry, tuple):
            cache = os.environ.get("VIDEOPRISM_CACHE_DIR", "")
            candidate = os.path.join(cache, entry[1]) if cache else ""
            if not candidate or not os.path.exists(candidate):
                raise FileNotFoundError(
                    f"{entry[1]} (Hugging Face repo {entry[0]}) is not available locally; pass "
                    "checkpoint_path= or set VIDEOPRISM_CACHE_DIR (no network download here)")
            checkpoint_path = candidate
        else:
            checkpoint_path = entry
    return utils.load_checkpoint(checkpoint_path)


def load_text_tokenizer(name: str):
    if name not in TEXT_TOKENIZERS:
        raise ValueError(f"Text tokenizer `{name}` not found.")
    raise NotImplementedError("text tokenizers are out of scope for the video-encoder path")
