"""Second, independent CPU restatement of the FactorizedEncoder forward in plain PyTorch
(fp64) — test infrastructure used only to cross-check the NumPy oracle.

Written from the reference's module semantics (encoders.py:411-580, layers.py:208-872)
with torch primitives (F.layer_norm, torch.erf, torch.softmax, einsum) instead of the
oracle's NumPy code, so that a shared misreading would have to be made twice.
"""

import torch
import torch.nn.functional as F


def _t(x):
    return torch.as_tensor(x, dtype=torch.float64)


def _ln(x, p):
    d = x.shape[-1]
    return F.layer_norm(x, (d,), weight=_t(p["scale"]) + 1.0, bias=_t(p["bias"]), eps=1e-6)


def _stack(x, st, L, heads, cap, paddings):
    xl = st["x_layers"]
    B, S, D = x.shape
    dh = D // heads
    if paddings is not None:
        pad = torch.as_tensor(paddings, dtype=torch.float64)
    else:
        pad = torch.zeros(B, S, dtype=torch.float64)
    masked = pad[:, None, None, :] > 0.5
    all_masked = masked.all(dim=-1, keepdim=True)
    for i in range(L):
        sa = xl["self_attention"]
        h = F.layer_norm(x, (D,), weight=_t(xl["layer_norm"]["scale"][i]) + 1.0,
                         bias=_t(xl["layer_norm"]["bias"][i]), eps=1e-6)
        q = torch.einsum("bsd,dnh->bsnh", h, _t(sa["query"]["w"][i])) + _t(sa["query"]["b"][i])
        k = torch.einsum("bsd,dnh->bsnh", h, _t(sa["key"]["w"][i])) + _t(sa["key"]["b"][i])
        v = torch.einsum("bsd,dnh->bsnh", h, _t(sa["value"]["w"][i])) + _t(sa["value"]["b"][i])
        q = q / dh ** 0.5
        logits = torch.einsum("btnh,bsnh->bnts", q, k)
        logits = cap * torch.tanh(logits / cap)
        # masked keys drop out; a row whose keys are all masked attends uniformly
        logits = torch.where(masked & ~all_masked, torch.full_like(logits, -1e300), logits)
        logits = torch.where(all_masked.expand_as(logits), torch.zeros_like(logits), logits)
        probs = torch.softmax(logits, dim=-1)
        enc = torch.einsum("bnts,bsnh->btnh", probs, v)
        att = torch.einsum("btnh,dnh->btd", enc, _t(sa["post"]["w"][i])) + _t(sa["post"]["b"][i])
        x = x + att
        ff = xl["ff_layer"]
        y = F.layer_norm(x, (D,), weight=_t(ff["layer_norm"]["scale"][i]) + 1.0,
                         bias=_t(ff["layer_norm"]["bias"][i]), eps=1e-6)
        a = y @ _t(ff["ffn_layer1"]["linear"]["kernel"][i]) + _t(ff["ffn_layer1"]["linear"]["bias"][i])
        a = 0.5 * a * (1.0 + torch.erf(a / 2 ** 0.5))
        a = a * (1.0 - pad[..., None])
        o = a @ _t(ff["ffn_layer2"]["linear"]["kernel"][i]) + _t(ff["ffn_layer2"]["linear"]["bias"][i])
        o = o * (1.0 - pad[..., None])
        x = x + o
    return x


def _resize(emb, out_len):
    """jax.image.resize(..., 'bilinear') along axis 0: for upsampling the half-pixel
    linear interpolation with edge clamp of encoders_mlx.py:104-137; for downsampling a
    triangle filter stretched by in/out (antialias), each output normalised to sum 1."""
    n = emb.shape[0]
    if out_len >= n:
        coords = (torch.arange(out_len, dtype=torch.float64) + 0.5) * (n / out_len) - 0.5
        lo = torch.floor(coords)
        wu = torch.clamp(coords - lo, 0.0, 1.0)
        li = torch.clamp(lo.long(), 0, n - 1)
        ui = torch.clamp(lo.long() + 1, 0, n - 1)
        return emb[li] * (1 - wu)[:, None] + emb[ui] * wu[:, None]
    ratio = n / out_len
    centres = (torch.arange(out_len, dtype=torch.float64) + 0.5) * ratio - 0.5
    src = torch.arange(n, dtype=torch.float64)
    wts = torch.clamp(1.0 - (src[None, :] - centres[:, None]).abs() / ratio, min=0.0)
    wts = wts / wts.sum(dim=1, keepdim=True)
    return wts @ emb


def _resize_2d(emb, src_hw, dst_hw):
    d = emb.shape[-1]
    e = emb.reshape(src_hw[0], src_hw[1], d)
    e = _resize(e.reshape(src_hw[0], -1), dst_hw[0]).reshape(dst_hw[0], src_hw[1], d)
    e = _resize(e.permute(1, 0, 2).reshape(src_hw[1], -1), dst_hw[1])
    return e.reshape(dst_hw[1], dst_hw[0], d).permute(1, 0, 2).reshape(dst_hw[0] * dst_hw[1], d)


def factorized_encoder(params, video, cfg, frame_paddings=None):
    P, D = cfg["patch_size"], cfg["model_dim"]
    heads, cap = cfg["num_heads"], cfg["atten_logit_cap"]
    x = _t(video)
    b, t, h, w, c = x.shape
    m, n = h // P, w // P
    patches = x.reshape(b * t, m, P, n, P, c).permute(0, 1, 3, 2, 4, 5).reshape(b * t, m * n, P * P * c)
    pp = params["patch_projection"]["linear"]
    feats = patches @ _t(pp["kernel"]) + _t(pp["bias"])
    pe = _t(params["spatial_pos_emb"]["emb_var"])
    src_hw = tuple(cfg["pos_emb_shape"][-2:])
    pe = pe[: src_hw[0] * src_hw[1]]
    if src_hw != (m, n):
        pe = _resize_2d(pe, src_hw, (m, n))
    feats = feats + pe[None]
    sp_pad = None
    tp_pad = None
    if frame_paddings is not None:
        fp = _t(frame_paddings)
        sp_pad = fp.reshape(b * t, 1).expand(b * t, m * n)
        tp_pad = fp[:, None, :].expand(b, m * n, t).reshape(b * m * n, t)
    feats = _stack(feats, params["spatial_encoder"]["transformers_stack"], cfg["num_spatial_layers"],
                   heads, cap, sp_pad)
    feats = _ln(feats, params["spatial_ln"])
    spatial = feats.reshape(b, t * m * n, D)
    feats = feats.reshape(b, t, m * n, D).permute(0, 2, 1, 3).reshape(b * m * n, t, D)
    temb = _t(params["temporal_pos_emb"]["emb_var"])
    if temb.shape[0] != t:
        temb = _resize(temb, t)
    feats = feats + temb[None]
    feats = _stack(feats, params["temporal_encoder"]["transformers_stack"], cfg["num_temporal_layers"],
                   heads, cap, tp_pad)
    feats = _ln(feats, params["temporal_ln"])
    out = feats.reshape(b, m * n, t, D).permute(0, 2, 1, 3).reshape(b, t * m * n, D)
    return out.numpy(), spatial.numpy()


# ----------------------------------------------------------------------------------------
# LvT video-text model (encoders.py:656-910, layers.py:92-179, :502-527, :1044-1136)
# ----------------------------------------------------------------------------------------
def _stack_general(x, st, L, heads, cap, paddings, causal, act):
    """Pre-LN stack with the merged causal/padding mask: key s is visible to query t iff
    neither is padded and s <= t; a query with no visible key attends uniformly."""
    xl = st["x_layers"]
    B, S, D = x.shape
    dh = D // heads
    pad = torch.zeros(B, S, dtype=torch.float64) if paddings is None else _t(paddings)
    keyok = pad[:, None, :] < 0.5                                   # [B, 1, S]
    if causal:
        qok = pad[:, :, None] < 0.5                                 # [B, S, 1]
        tri = torch.tril(torch.ones(S, S, dtype=torch.bool))[None]  # s <= t
        visible = keyok & qok & tri                                 # [B, T, S]
    else:
        visible = keyok.expand(B, S, S)
    visible = visible[:, None]                                      # [B, 1, T, S]
    none = ~visible.any(dim=-1, keepdim=True)
    for i in range(L):
        sa = xl["self_attention"]
        h = F.layer_norm(x, (D,), weight=_t(xl["layer_norm"]["scale"][i]) + 1.0,
                         bias=_t(xl["layer_norm"]["bias"][i]), eps=1e-6)
        q = torch.einsum("bsd,dnh->bsnh", h, _t(sa["query"]["w"][i])) + _t(sa["query"]["b"][i])
        k = torch.einsum("bsd,dnh->bsnh", h, _t(sa["key"]["w"][i])) + _t(sa["key"]["b"][i])
        v = torch.einsum("bsd,dnh->bsnh", h, _t(sa["value"]["w"][i])) + _t(sa["value"]["b"][i])
        logits = torch.einsum("btnh,bsnh->bnts", q / dh ** 0.5, k)
        if cap > 0:
            logits = cap * torch.tanh(logits / cap)
        logits = torch.where(visible | none, logits, torch.full_like(logits, -torch.inf))
        logits = torch.where(none.expand_as(logits), torch.zeros_like(logits), logits)
        enc = torch.einsum("bnts,bsnh->btnh", torch.softmax(logits, dim=-1), v)
        x = x + torch.einsum("btnh,dnh->btd", enc, _t(sa["post"]["w"][i])) + _t(sa["post"]["b"][i])
        ff = xl["ff_layer"]
        y = F.layer_norm(x, (D,), weight=_t(ff["layer_norm"]["scale"][i]) + 1.0,
                         bias=_t(ff["layer_norm"]["bias"][i]), eps=1e-6)
        a = act(y @ _t(ff["ffn_layer1"]["linear"]["kernel"][i]) + _t(ff["ffn_layer1"]["linear"]["bias"][i]))
        a = a * (1.0 - pad[..., None])
        o = a @ _t(ff["ffn_layer2"]["linear"]["kernel"][i]) + _t(ff["ffn_layer2"]["linear"]["bias"][i])
        x = x + o * (1.0 - pad[..., None])
    return x


def _gelu(a):
    return 0.5 * a * (1.0 + torch.erf(a / 2 ** 0.5))


def pooler(tokens, p, heads, hidden=None):
    """AttenTokenPoolingLayer: one learned query, dh = hidden/heads (4D for the CLIP pooler, D for
    the classifier's), per-dim scale, no cap, LN."""
    x = _t(tokens)
    D = x.shape[-1]
    pa = p["pooling_attention"]
    dh = (hidden or 4 * D) // heads
    q = torch.einsum("d,dnh->nh", _t(p["pooling_attention_query"])[0], _t(pa["query"]["w"]))
    q = (q + _t(pa["query"]["b"])) * (1.442695041 / dh ** 0.5) * F.softplus(_t(pa["per_dim_scale"]["per_dim_scale"]))
    k = torch.einsum("bsd,dnh->bsnh", x, _t(pa["key"]["w"])) + _t(pa["key"]["b"])
    v = torch.einsum("bsd,dnh->bsnh", x, _t(pa["value"]["w"])) + _t(pa["value"]["b"])
    probs = torch.softmax(torch.einsum("nh,bsnh->bns", q, k), dim=-1)
    enc = torch.einsum("bns,bsnh->bnh", probs, v)
    out = torch.einsum("bnh,dnh->bd", enc, _t(pa["post"]["w"])) + _t(pa["post"]["b"])
    return _ln(out, p["pooling_attention_layer_norm"])


def _l2n(x):
    return x / torch.sqrt((x * x).sum(-1, keepdim=True) + 1e-12)


def video_clip(params, cfg, video, ids, paddings, frame_paddings=None):
    """-> (video_emb, text_emb, frame_emb), all L2-normalised, fp64 numpy."""
    D, heads, cap = cfg["model_dim"], cfg["num_heads"], cfg["atten_logit_cap"]
    vcfg = dict(cfg)
    feats, _ = factorized_encoder(params["vision_encoder"], video, vcfg, frame_paddings)
    x = _t(feats)
    if cfg["num_auxiliary_layers"]:
        x = _stack_general(x, params["auxiliary_encoder"]["transformers_stack"], cfg["num_auxiliary_layers"],
                           heads, cap, None, False, _gelu)
    pp = params["contrastive_vision_pooler"]
    vemb = _l2n(pooler(x, pp, heads))
    b, t = video.shape[:2]
    femb = _l2n(pooler(x.reshape(b * t, -1, D), pp, heads)).reshape(b, t, D)
    te = params["text_encoder"]
    idt = torch.as_tensor(ids, dtype=torch.long)
    Q, L = idt.shape
    emb = _t(te["token_emb"]["emb_var"])[idt.clamp(0, cfg["vocabulary_size"] - 1)] * D ** 0.5
    pos = torch.arange(L, dtype=torch.float64)[:, None]
    inv = torch.exp(torch.arange(D // 2, dtype=torch.float64) * -(torch.log(torch.tensor(1e4, dtype=torch.float64))
                                                                  / max(D // 2 - 1, 1)))
    emb = emb + torch.cat([torch.sin(pos * inv), torch.cos(pos * inv)], dim=-1)[None]
    cls = _t(te["cls_emb"]).expand(Q, 1, D) * D ** 0.5
    y = torch.cat([emb, cls], dim=1)
    pad = torch.cat([_t(paddings), torch.zeros(Q, 1, dtype=torch.float64)], dim=1)
    y = _stack_general(y, te["unimodal_transformer"], cfg["num_unimodal_layers"], heads, cap, pad,
                       cfg["enable_causal_atten"], torch.relu)
    temb = _l2n(_ln(y, te["unimodal_ln"])[:, -1])
    return vemb.numpy(), temb.numpy(), femb.numpy()


def video_classifier(params, cfg, video):
    """encoders.py:583-653 -> logits (fp64 numpy)."""
    feats, _ = factorized_encoder(params["encoder"], video, cfg)
    emb = pooler(_t(feats), params["atten_pooler"], cfg["num_heads"], hidden=cfg["model_dim"])
    proj = params["projection"]["linear"]
    return (emb @ _t(proj["kernel"]) + _t(proj["bias"])).numpy()
