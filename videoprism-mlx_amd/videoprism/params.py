"""Parameter trees in the reference's Flax layout (scanned layers, leading L axis).

Leaf names/shapes follow what `FactorizedEncoder(scan=True).init(...)` creates
(encoders.py:391-580, layers.py:208-499, :940-1041): 40 leaves for any config
(encoders_test.py:170), keys '/'-joined under 'params' (utils.py:84-105).

Also converts the MLX-side files written by the reference's convert_weights.py
(unstacked `.../layers/{i}/...`, kernel/scale/emb_var renamed to `weight`,
convert_weights.py:88-104, :165-202) back to this canonical layout.
"""

from __future__ import annotations

import math
import re
from typing import Iterable

import numpy as np

_LAYER_LEAVES = (
    ("layer_norm/scale", ("D",)),
    ("layer_norm/bias", ("D",)),
    ("self_attention/query/w", ("D", "N", "H")),
    ("self_attention/query/b", ("N", "H")),
    ("self_attention/key/w", ("D", "N", "H")),
    ("self_attention/key/b", ("N", "H")),
    ("self_attention/value/w", ("D", "N", "H")),
    ("self_attention/value/b", ("N", "H")),
    ("self_attention/post/w", ("D", "N", "H")),
    ("self_attention/post/b", ("D",)),
    ("ff_layer/layer_norm/scale", ("D",)),
    ("ff_layer/layer_norm/bias", ("D",)),
    ("ff_layer/ffn_layer1/linear/kernel", ("D", "F")),
    ("ff_layer/ffn_layer1/linear/bias", ("F",)),
    ("ff_layer/ffn_layer2/linear/kernel", ("F", "D")),
    ("ff_layer/ffn_layer2/linear/bias", ("D",)),
)


def encoder_leaf_specs(cfg: dict, scan: bool = True) -> dict[str, tuple[int, ...]]:
    """Flat {path: shape} of a FactorizedEncoder's params for a CONFIGS entry."""
    D = cfg["model_dim"]
    nh = cfg["num_heads"]
    dims = {"D": D, "N": nh, "H": D // nh, "F": cfg["mlp_dim"]}
    P = cfg["patch_size"]
    pt, ph, pw = cfg["pos_emb_shape"]
    specs = {
        "patch_projection/linear/kernel": (P * P * 3, D),
        "patch_projection/linear/bias": (D,),
        "spatial_pos_emb/emb_var": (ph * pw, D),
    }
    for stack, L in (("spatial_encoder", cfg["num_spatial_layers"]),
                     ("temporal_encoder", cfg["num_temporal_layers"])):
        for name, shp in _LAYER_LEAVES:
            shape = tuple(dims[s] for s in shp)
            if scan:
                specs[f"{stack}/transformers_stack/x_layers/{name}"] = (L,) + shape
            else:
                for i in range(L):
                    specs[f"{stack}/transformers_stack/x_layers_{i}/{name}"] = shape
        if stack == "spatial_encoder":
            specs["spatial_ln/scale"] = (D,)
            specs["spatial_ln/bias"] = (D,)
            specs["temporal_pos_emb/emb_var"] = (pt, D)
    specs["temporal_ln/scale"] = (D,)
    specs["temporal_ln/bias"] = (D,)
    return specs


def _stack_specs(prefix: str, L: int, dims: dict, scan: bool) -> dict:
    out = {}
    for name, shp in _LAYER_LEAVES:
        shape = tuple(dims[s] for s in shp)
        if scan:
            out[f"{prefix}/x_layers/{name}"] = (L,) + shape
        else:
            for i in range(L):
                out[f"{prefix}/x_layers_{i}/{name}"] = shape
    return out


def clip_leaf_specs(cfg: dict, scan: bool = True) -> dict[str, tuple[int, ...]]:
    """Flat {path: shape} of a FactorizedVideoCLIP (encoders.py:762-910) for a CONFIGS
    'videoprism_lvt_*' entry plus `vocabulary_size`: the vision encoder under
    'vision_encoder/', the auxiliary ViT (:846-857), the contrastive pooler
    (layers.py:1044-1136, hidden 4D so dim_per_head = 4D/N) and the text tower
    (:656-759, mlp_dim = 4D, :895).  88 leaves scanned / 136 unrolled for the reference's
    tiny test config (encoders_test.py:339)."""
    D = cfg["model_dim"]
    nh = cfg["num_heads"]
    specs = {f"vision_encoder/{k}": v for k, v in encoder_leaf_specs(cfg, scan).items()}
    La = cfg.get("num_auxiliary_layers", 0)
    if La > 0:
        specs.update(_stack_specs("auxiliary_encoder/transformers_stack", La,
                                  {"D": D, "N": nh, "H": D // nh, "F": cfg["mlp_dim"]}, scan))
    dp = 4 * D // nh
    pre = "contrastive_vision_pooler"
    specs[f"{pre}/pooling_attention_query"] = (1, D)
    specs[f"{pre}/pooling_attention/per_dim_scale/per_dim_scale"] = (dp,)
    for q in ("query", "key", "value"):
        specs[f"{pre}/pooling_attention/{q}/w"] = (D, nh, dp)
        specs[f"{pre}/pooling_attention/{q}/b"] = (nh, dp)
    specs[f"{pre}/pooling_attention/post/w"] = (D, nh, dp)
    specs[f"{pre}/pooling_attention/post/b"] = (D,)
    specs[f"{pre}/pooling_attention_layer_norm/scale"] = (D,)
    specs[f"{pre}/pooling_attention_layer_norm/bias"] = (D,)
    specs["text_encoder/token_emb/emb_var"] = (cfg["vocabulary_size"], D)
    specs["text_encoder/cls_emb"] = (1, 1, D)
    specs.update(_stack_specs("text_encoder/unimodal_transformer", cfg["num_unimodal_layers"],
                              {"D": D, "N": nh, "H": D // nh, "F": 4 * D}, scan))
    specs["text_encoder/unimodal_ln/scale"] = (D,)
    specs["text_encoder/unimodal_ln/bias"] = (D,)
    return specs


def classifier_leaf_specs(cfg: dict, num_classes: int, scan: bool = True) -> dict[str, tuple[int, ...]]:
    """FactorizedVideoClassifier (encoders.py:583-653): 'encoder/...', 'atten_pooler/...'
    (AttenTokenPoolingLayer, hidden D so dim_per_head = D/N) and 'projection/linear/...':
    54 leaves for a scanned encoder (encoders_test.py:224)."""
    D = cfg["model_dim"]
    nh = cfg["num_heads"]
    dp = D // nh
    specs = {f"encoder/{k}": v for k, v in encoder_leaf_specs(cfg, scan).items()}
    pre = "atten_pooler"
    specs[f"{pre}/pooling_attention_query"] = (1, D)
    specs[f"{pre}/pooling_attention/per_dim_scale/per_dim_scale"] = (dp,)
    for q in ("query", "key", "value"):
        specs[f"{pre}/pooling_attention/{q}/w"] = (D, nh, dp)
        specs[f"{pre}/pooling_attention/{q}/b"] = (nh, dp)
    specs[f"{pre}/pooling_attention/post/w"] = (D, nh, dp)
    specs[f"{pre}/pooling_attention/post/b"] = (D,)
    specs[f"{pre}/pooling_attention_layer_norm/scale"] = (D,)
    specs[f"{pre}/pooling_attention_layer_norm/bias"] = (D,)
    specs["projection/linear/kernel"] = (D, num_classes)
    specs["projection/linear/bias"] = (num_classes,)
    return specs


def count_params(specs: dict[str, tuple[int, ...]]) -> int:
    return int(sum(int(np.prod(s)) for s in specs.values()))


# ------------------------------------------------------------------------------------ #
# tree helpers (utils.py:84-105 recover_tree and its inverse)
# ------------------------------------------------------------------------------------ #
def flatten(tree: dict, prefix: str = "") -> dict[str, np.ndarray]:
    out = {}
    for k, v in tree.items():
        key = f"{prefix}/{k}" if prefix else str(k)
        if isinstance(v, dict):
            out.update(flatten(v, key))
        else:
            out[key] = v
    return out


def unflatten(flat: dict) -> dict:
    tree: dict = {}
    for key, v in flat.items():
        node = tree
        parts = key.split("/")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = v
    return tree


def canonical_params(variables) -> dict[str, np.ndarray]:
    """Accepts {'params': tree}, a bare tree, or a flat '/'-keyed dict (Flax repeated npz,
    optionally prefixed by 'params/', or MLX-converted unstacked keys); returns the flat
    scanned Flax layout as fp32 numpy arrays."""
    if isinstance(variables, dict) and "params" in variables and isinstance(variables["params"], dict):
        variables = variables["params"]
    flat = {}
    for k, v in (flatten(variables) if any(isinstance(x, dict) for x in variables.values())
                 else dict(variables)).items():
        k = k[len("params/"):] if k.startswith("params/") else k
        flat[k] = v
    if any(re.search(r"/layers/\d+/", k) for k in flat) or any(re.search(r"/x_layers_\d+/", k) for k in flat):
        flat = _restack(flat)
    elif any(k.endswith("/weight") for k in flat):  # renamed but still stacked
        flat = {_mlx_rename(k): v for k, v in flat.items()}
    return {k: _to_f32(v) for k, v in flat.items()}


def _to_f32(v) -> np.ndarray:
    try:
        import torch
        if isinstance(v, torch.Tensor):
            return v.detach().float().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32))


# inverse of convert_weights.py:88-104 rename_parameter ('/kernel', '/scale', '/emb_var' ->
# '/weight'), by leaf; token_emb is the one the reference's own loader maps back explicitly
# (weight_utils.py:33-34)
_MLX_RENAMES = (
    ("patch_projection/linear/weight", "patch_projection/linear/kernel"),
    ("pos_emb/weight", "pos_emb/emb_var"),
    ("token_emb/weight", "token_emb/emb_var"),
    ("linear/weight", "linear/kernel"),
    ("layer_norm/weight", "layer_norm/scale"),
    ("_ln/weight", "_ln/scale"),
)


def _mlx_rename(k: str) -> str:
    for a, b in _MLX_RENAMES:
        if k.endswith(a):
            return k[: -len(a)] + b
    return k


def _restack(flat: dict) -> dict:
    """Unstacked layers (`.../layers/{i}/...` from convert_weights.py:165-202, or Flax
    unrolled `x_layers_{i}`) -> scanned `.../x_layers/...` with a leading L axis."""
    groups: dict[tuple[str, str], dict[int, np.ndarray]] = {}
    out = {}
    for k, v in flat.items():
        k = _mlx_rename(k)
        m = re.match(r"^(.*)/(?:layers/(\d+)|x_layers_(\d+))/(.*)$", k)
        if m:
            idx = int(m.group(2) if m.group(2) is not None else m.group(3))
            groups.setdefault((m.group(1), m.group(4)), {})[idx] = np.asarray(v)
        else:
            out[k] = v
    for (stack, leaf), per in groups.items():
        n = max(per) + 1
        if sorted(per) != list(range(n)):
            raise ValueError(f"non-contiguous layer indices under {stack}: {sorted(per)}")
        out[f"{stack}/x_layers/{leaf}"] = np.stack([per[i] for i in range(n)], axis=0)
    return out


def validate(flat: dict, specs: dict) -> None:
    missing = sorted(set(specs) - set(flat))
    if missing:
        raise ValueError(f"missing parameters: {missing[:5]}{' ...' if len(missing) > 5 else ''}")
    extra = sorted(set(flat) - set(specs))
    if extra:
        raise ValueError(f"unexpected parameters: {extra[:5]}{' ...' if len(extra) > 5 else ''}")
    for k, s in specs.items():
        if tuple(flat[k].shape) != tuple(s):
            raise ValueError(f"shape mismatch for {k}: expected {s}, got {tuple(flat[k].shape)}")


# ------------------------------------------------------------------------------------ #
# initialisers
# ------------------------------------------------------------------------------------ #
def synthetic_params(cfg: dict, seed: int = 0, specs: dict | None = None) -> dict:
    """Deterministic synthetic weights: kernels N(0, 1/fan_in), biases
    N(0, 0.02), LN scale N(0, 0.1) (used as 1+scale), positional embeddings N(0, 1/D).
    Non-zero biases/scales so that parity tests exercise every term.  Returns {'params': tree}."""
    rng = np.random.default_rng(seed)
    D = cfg["model_dim"]
    flat = {}
    for k, shape in (specs or encoder_leaf_specs(cfg)).items():
        leaf = k.rsplit("/", 1)[-1]
        if leaf == "pooling_attention_query":
            std = 1.0
        elif leaf == "cls_emb":
            std = 1.0 / math.sqrt(D)
        elif leaf in ("kernel", "w"):
            if k.endswith("post/w"):
                fan_in = shape[-2] * shape[-1]
            else:
                fan_in = shape[-3] if len(shape) >= 3 and k.endswith("/w") else shape[-2]
            std = 1.0 / math.sqrt(fan_in)
        elif leaf in ("scale", "per_dim_scale"):
            std = 0.1
        elif leaf == "emb_var":
            std = 1.0 / math.sqrt(D)
        else:
            std = 0.02
        flat[k] = rng.standard_normal(shape, dtype=np.float64).astype(np.float32) * np.float32(std)
    return {"params": unflatten(flat)}


def flax_default_init(cfg: dict, seed: int = 0) -> dict:
    """Distributions of Flax's initialisers for this module (layers.py:28 lecun_normal
    kernels, zero biases, LN scale 0 / bias 0, encoders.py:296-303 lecun pos-emb).  The
    JAX PRNG stream itself is not reproducible without JAX; numpy is used instead."""
    rng = np.random.default_rng(seed)
    flat = {}
    for k, shape in encoder_leaf_specs(cfg).items():
        leaf = k.rsplit("/", 1)[-1]
        base = shape[1:] if "x_layers/" in k else shape
        if leaf in ("kernel", "w", "emb_var"):
            if len(base) == 2:
                fan_in = base[0]
            else:  # [D, N, H]: in_axis=-2, out_axis=-1, receptive field D
                fan_in = base[-2] * int(np.prod(base[:-2]))
            std = math.sqrt(1.0 / fan_in) / 0.87962566103423978  # truncated normal
            v = rng.standard_normal(shape)
            v = np.clip(v, -2.0, 2.0) * std
            flat[k] = v.astype(np.float32)
        else:
            flat[k] = np.zeros(shape, np.float32)
    return {"params": unflatten(flat)}


def leaves(tree: dict) -> Iterable[np.ndarray]:
    return flatten(tree).values()
