"""CPU restatement of the VideoPrism FactorizedEncoder forward — TEST INFRASTRUCTURE ONLY.

This module is the parity checker for the MI355X HIP path.  Only `tests/`,
`__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py` may import it;
the product package (`videoprism-mlx_amd/videoprism`) never does, and the product
path fails loudly when its HIP library is missing instead of falling back here.

It restates, in plain NumPy (fp64 by default, fp32 on request, optional bf16
rounding emulation), the Flax reference at /root/reference/videoprism:

  * layers.py:31            gelu (exact erf)
  * layers.py:39-179        mask helpers (padding mask, -0.7*finfo.max fill)
  * layers.py:208-270       LayerNorm (biased var, eps 1e-6, scale+1, bias)
  * layers.py:273-313       FeedForward (Dense + activation)
  * layers.py:316-430       TransformerFeedForward (pre-LN, GELU, padding zeroing, residual)
  * layers.py:433-499       AttentionProjection (w[D,N,H]; q/k/v and 'post' einsums)
  * layers.py:530-746       DotProductAttention (q *= dh^-0.5, tanh cap, fp32 softmax)
  * layers.py:749-872       Transformer (pre-LN block)
  * layers.py:940-1041      StackedTransformer (scanned params, leading L axis)
  * encoders.py:70-104      _image_to_patch ('(m p)(n q) c -> (m n)(p q c)')
  * encoders.py:107-165     _interpolate_emb_1d/2d (jax.image.resize 'bilinear')
  * encoders.py:269-307     TrainablePositionalEmbedding (slice of emb_var)
  * encoders.py:310-388     VisionTransformer
  * encoders.py:391-580     FactorizedEncoder.__call__ / encode_with_patches
  LvT video-text:
  * layers.py:92-179        causal mask, _merge_masks, compute_attention_masks_for_fprop
  * layers.py:502-527       PerDimScale (1.442695041/sqrt(dh) * softplus)
  * layers.py:1044-1136     AttenTokenPoolingLayer
  * encoders.py:50-67       _l2_normalize
  * encoders.py:168-266     Embedding (index, scale_sqrt_depth), PositionalEmbedding
  * encoders.py:656-759     TextEncoder (causal, ReLU, CLS token, unimodal_ln)
  * encoders.py:762-910     FactorizedVideoCLIP.__call__ (auxiliary encoder, pooler, L2)

PARITY UNPINNED: the reference's own tests pin only shapes and parameter-leaf
counts (encoders_test.py:170, models_test.py:52); JAX/Flax are not installed in
this container (ModuleNotFoundError, not a permission denial), no checkpoint is
available offline, and the reference ships no golden vectors for this path.  The
restatement is therefore pinned only by those structural facts, by a second
independent restatement (torch-CPU, tests/test_oracle.py) and by the golden
fixtures it generated itself (tests/golden/, script tests/golden/make_golden.py).
"""

from __future__ import annotations

import numpy as np
from scipy.special import erf as _erf

F32_MAX = float(np.finfo(np.float32).max)


# --------------------------------------------------------------------------- #
# numeric helpers
# --------------------------------------------------------------------------- #
def round_bf16(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even to bfloat16, returned as float32 (emulation)."""
    a = np.ascontiguousarray(x, dtype=np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return (u.astype(np.uint32) << 16).view(np.float32).reshape(a.shape)


class Numerics:
    """Where the Flax graph holds tensors in `fprop_dtype` (layers.py:182-205).

    mode 'f64'  : everything float64 (mathematical reference)
    mode 'f32'  : everything float32 (Flax fprop_dtype=float32)
    mode 'bf16' : float32 arithmetic, activations/params rounded to bf16 at the
                  points where Flax-bf16 stores bf16 (models.py:301-302); softmax
                  stays fp32 (layers.py:650-654).
    mode 'wbf16': float64 arithmetic on bf16-rounded parameters only: the part of the bf16
                  mode's deviation from fp64 that the parameter cast alone causes (not a
                  reference mode -- a parity-analysis tool).
    """

    def __init__(self, mode: str = "f64"):
        assert mode in ("f64", "f32", "bf16", "wbf16"), mode
        self.mode = mode
        self.dt = np.float32 if mode in ("f32", "bf16") else np.float64

    def act(self, x):
        x = np.asarray(x, dtype=self.dt)
        return round_bf16(x) if self.mode == "bf16" else x

    def param(self, p):
        if self.mode == "wbf16":
            return round_bf16(np.asarray(p, dtype=np.float64))
        return self.act(p)


# --------------------------------------------------------------------------- #
# layers.py
# --------------------------------------------------------------------------- #
def gelu(x):
    """layers.py:31 — jax.nn.gelu(approximate=False) = 0.5 x (1 + erf(x/sqrt 2))."""
    return 0.5 * x * (1.0 + _erf(x / np.sqrt(2.0)))


def layer_norm(x, scale, bias, nm: Numerics, eps: float = 1e-6):
    """layers.py:208-270 (direct_scale=False, reductions_in_fp32=False)."""
    mean = nm.act(np.mean(x, axis=-1, keepdims=True))
    xc = nm.act(x - mean)
    var = nm.act(np.mean(nm.act(xc * xc), axis=-1, keepdims=True))
    normed = nm.act(xc * nm.act(1.0 / np.sqrt(var + eps)))
    normed = nm.act(normed * nm.act(nm.param(scale) + 1.0))
    return nm.act(normed + nm.param(bias))


def dense(x, kernel, bias, nm: Numerics):
    """layers.py:273-313 — nn.Dense(x @ kernel + bias), params cast to fprop dtype."""
    y = nm.act(np.matmul(x, nm.param(kernel)))
    return nm.act(y + nm.param(bias))


def attention_projection_in(x, w, b, nm: Numerics):
    """layers.py:455-499, is_output_projection=False: '...D,DNH->...NH' + b[N,H]."""
    d, n, h = w.shape
    y = nm.act(np.matmul(x, nm.param(w).reshape(d, n * h)))
    y = y.reshape(*x.shape[:-1], n, h)
    return nm.act(y + nm.param(b))


def attention_projection_out(enc, w, b, nm: Numerics):
    """layers.py:455-499, is_output_projection=True: '...NH,DNH->...D' + b[D]."""
    d, n, h = w.shape
    flat = enc.reshape(*enc.shape[:-2], n * h)
    y = nm.act(np.matmul(flat, nm.param(w).reshape(d, n * h).T))
    return nm.act(y + nm.param(b))


def padding_mask(paddings):
    """layers.py:75-89 — paddings[:,None,None,:] * (-0.7*finfo.max); 0 means keep."""
    return paddings[:, None, None, :].astype(np.float64) * (-0.7 * F32_MAX)


def apply_mask_to_logits(logits, mask):
    """layers.py:51-72 — where(mask >= 0.5*min, logits, min), min = -0.7*f32max."""
    min_value = -0.7 * F32_MAX
    return np.where(mask >= 0.5 * min_value, logits, min_value)


def softmax(x):
    """jax.nn.softmax over the last axis (max-subtracted)."""
    m = np.max(x, axis=-1, keepdims=True)
    e = np.exp(x - m)
    return e / np.sum(e, axis=-1, keepdims=True)


def dot_atten(q, k, v, mask, nm: Numerics, cap: float, dim_per_head: int):
    """layers.py:601-661 with _scale_query :569-584 and _cap_logits :586-594.

    q,k,v: [B, S, N, H]; mask: [B|1, 1, 1, S] (or None for all-valid).
    """
    q = nm.act(q * nm.act(dim_per_head ** -0.5))          # per_dim_scale disabled
    B, T, N, _ = q.shape
    S = k.shape[1]
    qc = max(1, _ATTN_CHUNK_ELEMS // max(1, B * N * S))
    if qc < T:
        # every query row's softmax is independent of the others: long sequences (the LvT
        # auxiliary encoder at T*N = 10240 tokens) run in query blocks so the [B, N, T, S]
        # logits never exist at once -- the same elementwise operations per row
        def rows(m, i):
            return m if m is None or m.shape[-2] == 1 else m[..., i:i + qc, :]
        return np.concatenate([_dot_atten_rows(q[:, i:i + qc], k, v, rows(mask, i), nm, cap)
                               for i in range(0, T, qc)], axis=1)
    return _dot_atten_rows(q, k, v, mask, nm, cap)


_ATTN_CHUNK_ELEMS = 1 << 27   # logits elements per query block (1 GiB in fp64)


def _dot_atten_rows(q, k, v, mask, nm: Numerics, cap: float):
    """dot_atten's body after _scale_query, for a block of (already scaled) query rows."""
    qt = np.transpose(q, (0, 2, 1, 3))                      # B N T H
    kt = np.transpose(k, (0, 2, 3, 1))                      # B N H S
    logits = nm.act(np.matmul(qt, kt))                      # 'BTNH,BSNH->BNTS'
    if cap and cap > 0.0:
        capv = nm.act(cap)
        logits = nm.act(capv * nm.act(np.tanh(nm.act(logits / capv))))
    sm_dt = np.float64 if nm.mode in ("f64", "wbf16") else np.float32  # softmax always >= fp32
    logits = logits.astype(sm_dt)
    if mask is not None:
        logits = apply_mask_to_logits(logits, mask).astype(sm_dt)
    probs = nm.act(softmax(logits))
    vt = np.transpose(v, (0, 2, 1, 3))                      # B N S H
    enc = nm.act(np.matmul(probs, vt))                      # B N T H
    return np.transpose(enc, (0, 2, 1, 3))                  # B T N H


def transformer_layer(x, p, paddings, mask, nm: Numerics, num_heads: int, cap: float):
    """layers.py:796-872 (norm_policy='pre', GELU, per-dim-scale off) for one layer.

    `p` is the per-layer slice of the scanned 'x_layers' subtree.
    """
    return transformer_layer_act(x, p, paddings, mask, nm, num_heads, cap, gelu)


def _layer_slice(tree, i):
    if isinstance(tree, dict):
        return {k: _layer_slice(v, i) for k, v in tree.items()}
    return tree[i]


def stacked_transformer(x, paddings, stack, nm: Numerics, num_layers: int,
                        num_heads: int, cap: float):
    """layers.py:990-1041 + Repeat(scan) :875-937 (params stacked on axis 0)."""
    if paddings is None:
        paddings = np.zeros(x.shape[:-1])
    mask = padding_mask(paddings)
    if not np.any(paddings):
        mask = None                                         # exact no-op (mask == 0)
    xl = stack["x_layers"]
    for i in range(num_layers):
        x = transformer_layer(x, _layer_slice(xl, i), paddings, mask, nm, num_heads, cap)
    return x


# --------------------------------------------------------------------------- #
# encoders.py
# --------------------------------------------------------------------------- #
def image_to_patch(inputs, patch_size: int):
    """encoders.py:70-104 — '... (m p)(n q) c -> ... (m n)(p q c)'."""
    if inputs.ndim < 4:
        raise ValueError(f"Image should be formatted as 4D [B, H, W, C], Shape: {inputs.shape}")
    h, w, c = inputs.shape[-3:]
    if h % patch_size or w % patch_size:
        raise ValueError(f"Image height ({h}) and width ({w}) should be multiples "
                         f"of patch_size ({patch_size}).")
    m, n = h // patch_size, w // patch_size
    lead = inputs.shape[:-3]
    x = inputs.reshape(*lead, m, patch_size, n, patch_size, c)
    nl = len(lead)
    perm = list(range(nl)) + [nl, nl + 2, nl + 1, nl + 3, nl + 4]
    x = np.transpose(x, perm)
    return x.reshape(*lead, m * n, patch_size * patch_size * c)


def _resize_weights(in_size: int, out_size: int) -> np.ndarray:
    """jax.image.resize(method='bilinear', antialias=True) 1-D weight matrix.

    Restates jax/_src/image/scale.py `compute_weight_mat` (jax version unpinned by
    requirements.txt:5): triangle kernel, half-pixel centres, kernel widened by
    1/scale when downsampling, columns normalised, samples outside the input
    range zeroed.  Upsampling reduces to half-pixel linear with edge clamp, as
    restated independently at encoders_mlx.py:104-137.  Returns W [in, out].
    """
    scale = out_size / in_size
    inv_scale = 1.0 / scale
    kernel_scale = max(inv_scale, 1.0)
    sample_f = (np.arange(out_size) + 0.5) * inv_scale - 0.5
    x = np.abs(sample_f[None, :] - np.arange(in_size)[:, None]) / kernel_scale
    w = np.maximum(0.0, 1.0 - x)
    tot = np.sum(w, axis=0, keepdims=True)
    w = np.where(np.abs(tot) > 1000.0 * float(np.finfo(np.float32).eps),
                 w / np.where(tot != 0, tot, 1), 0.0)
    inside = (sample_f >= -0.5) & (sample_f <= in_size - 0.5)
    return np.where(inside[None, :], w, 0.0)


def interpolate_emb_1d(emb, target_len: int):
    """encoders.py:107-130 — emb [1, N, D] -> [1, target_len, D]."""
    if emb.ndim > 3 or emb.shape[0] != 1:
        raise ValueError("The shape of the embedding should be (1, N, D)")
    wt = _resize_weights(emb.shape[1], target_len)          # [N, T']
    return np.einsum("nd,nt->td", emb[0], wt)[None]


def interpolate_emb_2d(emb, source_shape, target_shape):
    """encoders.py:133-165 — emb [1, H1*W1, D] -> [1, H2*W2, D] (separable bilinear)."""
    if emb.ndim > 3 or emb.shape[0] != 1:
        raise ValueError("The shape of the embedding should be (1, H * W, D)")
    if emb.shape[-2] != source_shape[0] * source_shape[1]:
        raise ValueError("The shape of the embedding does NOT match input specs.")
    d = emb.shape[-1]
    e = emb[0].reshape(source_shape[0], source_shape[1], d)
    wh = _resize_weights(source_shape[0], target_shape[0])
    ww = _resize_weights(source_shape[1], target_shape[1])
    out = np.einsum("hwd,hi,wj->ijd", e, wh, ww)
    return out.reshape(1, target_shape[0] * target_shape[1], d)


def _contains(collection, key):
    """encoders.py:36-47."""
    return collection if isinstance(collection, bool) else key in collection


def factorized_encoder(params, inputs, cfg: dict, mode: str = "f64",
                       frame_paddings=None, return_intermediate=False):
    """encoders.py:411-580 — FactorizedEncoder.__call__ + encode_with_patches.

    params: the Flax tree *under* 'params' (scanned layout).  cfg: the CONFIGS
    entry (models.py:83-104).  Returns (embeddings [B, T*N, D], outputs dict).
    """
    nm = Numerics(mode)
    P = cfg["patch_size"]
    D = cfg["model_dim"]
    heads = cfg["num_heads"]
    cap = cfg.get("atten_logit_cap", 0.0)
    b, t, h, w, c = inputs.shape
    assert h == w                                           # :435
    x = nm.act(np.asarray(inputs).reshape(b * t, h, w, c))
    patches = image_to_patch(x, P)                          # [BT, N, P*P*C]
    patches_paddings = None
    if frame_paddings is not None:
        frame_paddings = np.asarray(frame_paddings, dtype=np.float64)
        assert frame_paddings.shape == (b, t)
        patches_paddings = np.repeat(frame_paddings.reshape(b * t)[:, None],
                                     patches.shape[1], axis=-1)

    pp = params["patch_projection"]["linear"]
    feats = dense(patches, pp["kernel"], pp["bias"], nm)    # :488-494
    sp_shape = tuple(cfg["pos_emb_shape"][-2:])
    sp_len = int(np.prod(sp_shape))
    sp_emb = np.asarray(params["spatial_pos_emb"]["emb_var"], dtype=np.float64)[:sp_len][None]
    grid = (h // P, w // P)
    if sp_shape != grid:
        sp_emb = interpolate_emb_2d(sp_emb, sp_shape, grid)
    feats = nm.act(feats + nm.param(sp_emb))                # :514

    feats = stacked_transformer(feats, patches_paddings,
                                params["spatial_encoder"]["transformers_stack"], nm,
                                cfg["num_spatial_layers"], heads, cap)
    feats = layer_norm(feats, params["spatial_ln"]["scale"], params["spatial_ln"]["bias"], nm)
    spatial_features = feats
    n = feats.shape[1]
    feats = feats.reshape(b, t, n, D).transpose(0, 2, 1, 3).reshape(b * n, t, D)  # :535
    temporal_paddings = None
    if patches_paddings is not None:
        temporal_paddings = patches_paddings.reshape(b, t, n).transpose(0, 2, 1).reshape(b * n, t)

    t_len = cfg["pos_emb_shape"][0]
    t_emb = np.asarray(params["temporal_pos_emb"]["emb_var"], dtype=np.float64)[:t_len][None]
    if t_len != t:
        t_emb = interpolate_emb_1d(t_emb, t)                # :551-552
    feats = nm.act(feats + nm.param(t_emb))

    feats = stacked_transformer(feats, temporal_paddings,
                                params["temporal_encoder"]["transformers_stack"], nm,
                                cfg["num_temporal_layers"], heads, cap)
    feats = layer_norm(feats, params["temporal_ln"]["scale"], params["temporal_ln"]["bias"], nm)
    feats = feats.reshape(b, n, t, D).transpose(0, 2, 1, 3).reshape(b, t * n, D)  # :570

    outputs = {}
    if _contains(return_intermediate, "spatial_features"):
        outputs["spatial_features"] = spatial_features.reshape(b, t * n, D)     # :575-578
    return feats, outputs


# --------------------------------------------------------------------------- #
# op-level restatements used by the kernel unit tests
# --------------------------------------------------------------------------- #
def capped_softmax_attention(q, k, v, cap: float, key_mask=None):
    """Per-problem attention used to check the HIP attention kernels.

    q,k,v: [P, S, dh] with q already scaled (layers.py:569-584).  Returns [P, S, dh].
    key_mask: optional [P, S] (1 = padded key).  Follows layers.py:586-661.
    """
    logits = np.matmul(q, np.swapaxes(k, -1, -2))
    if cap > 0:
        logits = cap * np.tanh(logits / cap)
    if key_mask is not None:
        logits = apply_mask_to_logits(logits, padding_mask(key_mask)[:, 0])
    return np.matmul(softmax(logits), v)


# --------------------------------------------------------------------------- #
# LvT video-text model (FactorizedVideoCLIP) — SURVEY.md §8(f) f1
# --------------------------------------------------------------------------- #
def relu(x):
    """jax.nn.relu — the text tower's activation (encoders.py:743, layers.py:34)."""
    return np.maximum(x, 0.0)


def causal_mask(t: int):
    """layers.py:92-108 — [1, 1, T, T], (row < col) * (-0.7*finfo.max)."""
    row = np.arange(t)[:, None]
    col = np.arange(t)[None, :]
    return ((row < col).astype(np.float64) * (-0.7 * F32_MAX))[None, None]


def merge_masks(a, b):
    """layers.py:111-152 — elementwise minimum; a [B,1,1,S] key mask is first expanded to
    [B,1,S,S] as min(query_mask, key_mask), so padded *queries* are fully masked too."""
    def expand_t(key_mask):
        return np.minimum(np.swapaxes(key_mask, -1, -2), key_mask)
    if a.shape[-2] != b.shape[-2]:
        if a.shape[-2] == 1:
            a = expand_t(a)
        else:
            b = expand_t(b)
    return np.minimum(a, b)


def attention_masks_for_fprop(paddings, causal: bool):
    """layers.py:155-179 compute_attention_masks_for_fprop."""
    mask = padding_mask(paddings)
    if causal:
        mask = merge_masks(mask, causal_mask(paddings.shape[-1]))
    return mask


def transformer_layer_act(x, p, paddings, mask, nm: Numerics, num_heads: int, cap: float,
                          activation=gelu):
    """transformer_layer with a configurable FFN activation (layers.py:316-430: GELU in the
    vision stacks, ReLU in the text tower)."""
    d = x.shape[-1]
    h = layer_norm(x, p["layer_norm"]["scale"], p["layer_norm"]["bias"], nm)
    sa = p["self_attention"]
    q = attention_projection_in(h, sa["query"]["w"], sa["query"]["b"], nm)
    k = attention_projection_in(h, sa["key"]["w"], sa["key"]["b"], nm)
    v = attention_projection_in(h, sa["value"]["w"], sa["value"]["b"], nm)
    enc = dot_atten(q, k, v, mask, nm, cap, d // num_heads)
    att = attention_projection_out(enc, sa["post"]["w"], sa["post"]["b"], nm)
    x = nm.act(att + x)
    ff = p["ff_layer"]
    y = layer_norm(x, ff["layer_norm"]["scale"], ff["layer_norm"]["bias"], nm)
    a = nm.act(activation(dense(y, ff["ffn_layer1"]["linear"]["kernel"],
                                ff["ffn_layer1"]["linear"]["bias"], nm)))
    pad = None if paddings is None else nm.act(1.0 - paddings[..., None])
    if pad is not None:
        a = nm.act(a * pad)
    o = dense(a, ff["ffn_layer2"]["linear"]["kernel"], ff["ffn_layer2"]["linear"]["bias"], nm)
    if pad is not None:
        o = nm.act(o * pad)
    return nm.act(x + o)


def stacked_transformer_causal(x, paddings, stack, nm: Numerics, num_layers: int,
                               num_heads: int, cap: float, causal: bool, activation=gelu):
    """layers.py:990-1041 with enable_causal_atten and activation_fn (text tower)."""
    if paddings is None:
        paddings = np.zeros(x.shape[:-1])
    mask = attention_masks_for_fprop(np.asarray(paddings, np.float64), causal)
    if not causal and not np.any(paddings):
        mask = None
    xl = stack["x_layers"]
    for i in range(num_layers):
        x = transformer_layer_act(x, _layer_slice(xl, i), paddings, mask, nm, num_heads, cap,
                                  activation)
    return x


def softplus(x):
    return np.logaddexp(0.0, x)


def atten_token_pooling(tokens, p, nm: Numerics, num_heads: int, hidden_dim: int):
    """layers.py:1044-1136 AttenTokenPoolingLayer(num_queries=1, add_layer_norm=True,
    per-dim scale on, no logit cap, paddings None) -> [B, 1, D].

    q = query param projected to [N, dh] (dh = hidden_dim / N) and scaled by
    1.442695041/sqrt(dh) * softplus(per_dim_scale) (layers.py:502-527); K, V projections of
    the tokens; fp32 softmax (layers.py:650-654); 'post' back to D; LayerNorm.
    """
    b = tokens.shape[0]
    pa = p["pooling_attention"]
    dh = hidden_dim // num_heads
    query = np.tile(nm.param(p["pooling_attention_query"])[None], (b, 1, 1))   # [B,1,D]
    q = attention_projection_in(query, pa["query"]["w"], pa["query"]["b"], nm)  # [B,1,N,dh]
    k = attention_projection_in(tokens, pa["key"]["w"], pa["key"]["b"], nm)
    v = attention_projection_in(tokens, pa["value"]["w"], pa["value"]["b"], nm)
    scale = nm.act(nm.act(1.442695041 / np.sqrt(dh)) *
                   nm.act(softplus(nm.param(pa["per_dim_scale"]["per_dim_scale"]))))
    q = nm.act(q * scale)
    qt = np.transpose(q, (0, 2, 1, 3))
    kt = np.transpose(k, (0, 2, 3, 1))
    logits = nm.act(np.matmul(qt, kt))
    sm_dt = np.float64 if nm.mode in ("f64", "wbf16") else np.float32
    probs = nm.act(softmax(logits.astype(sm_dt)))
    enc = nm.act(np.matmul(probs, np.transpose(v, (0, 2, 1, 3))))
    enc = np.transpose(enc, (0, 2, 1, 3))                                       # [B,1,N,dh]
    out = attention_projection_out(enc, pa["post"]["w"], pa["post"]["b"], nm)   # [B,1,D]
    ln = p["pooling_attention_layer_norm"]
    return layer_norm(out, ln["scale"], ln["bias"], nm)


def l2_normalize(x, eps: float = 1e-12):
    """encoders.py:50-67 — always in fp32 (fp64 here), x / sqrt(sum x^2 + eps)."""
    x = np.asarray(x, dtype=np.float64)
    return x / np.sqrt(np.sum(x * x, axis=-1, keepdims=True) + eps)


def sinusoidal_positions(seq_length: int, dim: int, min_timescale: float = 1.0,
                         max_timescale: float = 10_000.0):
    """encoders.py:190-224 PositionalEmbedding: [seq_length, dim] = [sin | cos] (+zero pad
    for odd dim), computed in fp32 by the reference (restated in fp64)."""
    position = np.arange(seq_length, dtype=np.float64)[:, None]
    num_ts = dim // 2
    log_inc = np.log(float(max_timescale) / float(min_timescale)) / max(num_ts - 1, 1)
    inv = min_timescale * np.exp(np.arange(num_ts, dtype=np.float64) * -log_inc)
    st = position * inv[None, :]
    emb = np.concatenate([np.sin(st), np.cos(st)], axis=-1)
    if dim % 2:
        emb = np.pad(emb, [[0, 0], [0, 1]])
    return emb


def text_encoder(params, ids, paddings, cfg: dict, nm: Numerics):
    """encoders.py:656-759 TextEncoder(num_class_tokens=1, causal, ReLU, per-dim scale off,
    cap) -> features [B, L+1, D] after unimodal_ln.  Embedding lookup 'index' style with
    scale_sqrt_depth (encoders.py:226-266); ids outside [0, V) clamp (JAX gather)."""
    D = cfg["model_dim"]
    ids = np.asarray(ids)
    b, n = ids.shape
    table = nm.param(params["token_emb"]["emb_var"])
    emb = table[np.clip(ids, 0, table.shape[0] - 1)]
    emb = nm.act(emb * nm.act(D ** 0.5))
    pos = nm.act(sinusoidal_positions(n, D))[None]
    feats = nm.act(emb + pos)
    cls = np.tile(nm.param(params["cls_emb"]), (b, 1, 1))
    cls = nm.act(cls * nm.act(D ** 0.5))
    feats = np.concatenate([feats, cls], axis=1)
    pad = np.concatenate([np.asarray(paddings, np.float64), np.zeros((b, 1))], axis=-1)
    feats = stacked_transformer_causal(feats, pad, params["unimodal_transformer"], nm,
                                       cfg["num_unimodal_layers"], cfg["num_heads"],
                                       cfg.get("atten_logit_cap", 0.0),
                                       cfg.get("enable_causal_atten", True), relu)
    ln = params["unimodal_ln"]
    return layer_norm(feats, ln["scale"], ln["bias"], nm)


def video_clip(params, cfg: dict, inputs=None, text_token_ids=None, text_paddings=None,
               mode: str = "f64", normalize: bool = True, return_intermediate=False,
               frame_paddings=None):
    """encoders.py:762-910 FactorizedVideoCLIP.__call__ -> (video_emb [B,D] | None,
    text_emb [B,D] | None, outputs).  `params` is the tree under 'params'; cfg a CONFIGS
    'videoprism_lvt_*' entry (models.py:116-160) plus vocabulary_size."""
    nm = Numerics(mode)
    D = cfg["model_dim"]
    heads = cfg["num_heads"]
    cap = cfg.get("atten_logit_cap", 0.0)
    video_emb = text_emb = None
    outputs = {}
    if inputs is not None:
        t = inputs.shape[-4]
        vcfg = {k: cfg[k] for k in ("patch_size", "pos_emb_shape", "model_dim", "num_spatial_layers",
                                    "num_temporal_layers", "num_heads", "mlp_dim",
                                    "atten_logit_cap")}
        feats, vout = factorized_encoder(params["vision_encoder"], inputs, vcfg, mode,
                                         frame_paddings, return_intermediate)
        outputs.update(vout)
        if _contains(return_intermediate, "spatiotemporal_features"):
            outputs["spatiotemporal_features"] = feats
        if cfg.get("num_auxiliary_layers", 0) > 0:
            feats = stacked_transformer_causal(
                feats, None, params["auxiliary_encoder"]["transformers_stack"], nm,
                cfg["num_auxiliary_layers"], heads, cap, False, gelu)       # :846-857
        pooler = params["contrastive_vision_pooler"]
        video_emb = atten_token_pooling(feats, pooler, nm, heads, 4 * D)[:, 0]
        if normalize:
            video_emb = l2_normalize(video_emb)
        if _contains(return_intermediate, "frame_embeddings"):
            b = feats.shape[0]
            n = feats.shape[1] // t
            ff = feats.reshape(b * t, n, D)                                  # :876
            fe = atten_token_pooling(ff, pooler, nm, heads, 4 * D)[:, 0].reshape(b, t, D)
            if normalize:
                fe = l2_normalize(fe)
            outputs["frame_embeddings"] = fe
    if text_token_ids is not None:
        assert text_paddings is not None, "Text paddings are required."
        tf = text_encoder(params["text_encoder"], text_token_ids, text_paddings, cfg, nm)
        text_emb = tf[:, -1]                                                 # :906
        if normalize:
            text_emb = l2_normalize(text_emb)
    return video_emb, text_emb, outputs


def masked_attention(q, k, v, cap: float, key_pad=None, causal: bool = False):
    """Op-level restatement for the generic masked attention kernel: q,k,v [P, S, dh] with q
    already scaled; mask = compute_attention_masks_for_fprop(key_pad, causal) (layers.py:155-179)
    applied as in _dot_atten (layers.py:643-661).  Returns [P, S, dh]."""
    logits = np.matmul(q, np.swapaxes(k, -1, -2))
    if cap > 0:
        logits = cap * np.tanh(logits / cap)
    pad = np.zeros(q.shape[:2]) if key_pad is None else np.asarray(key_pad, np.float64)
    mask = attention_masks_for_fprop(pad, causal)[:, 0]
    return np.matmul(softmax(apply_mask_to_logits(logits, mask)), v)


def video_classifier(params, cfg: dict, inputs, mode: str = "f64", return_intermediate=False,
                     frame_paddings=None):
    """encoders.py:583-653 FactorizedVideoClassifier.__call__ -> (logits [B, C], outputs).
    cfg: the encoder_params (a FactorizedEncoder CONFIGS entry).  The pooler is
    AttenTokenPoolingLayer(num_heads, hidden_dim=model_dim, num_queries=1) with its defaults
    (per-dim scale, LayerNorm), applied with paddings None."""
    nm = Numerics(mode)
    feats, outputs = factorized_encoder(params["encoder"], inputs, cfg, mode, frame_paddings,
                                        return_intermediate)
    if _contains(return_intermediate, "spatiotemporal_features"):
        outputs["spatiotemporal_features"] = feats
    emb = atten_token_pooling(feats, params["atten_pooler"], nm, cfg["num_heads"],
                              cfg["model_dim"])[:, 0]
    if _contains(return_intermediate, "global_embeddings"):
        outputs["global_embeddings"] = emb
    proj = params["projection"]["linear"]
    return dense(emb, proj["kernel"], proj["bias"], nm), outputs
