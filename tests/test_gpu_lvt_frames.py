"""The LvT video-text path and the >256-key attention at token counts that are not multiples of 256.

The reference's FactorizedVideoCLIP runs at any H = W divisible by the patch: the vision encoder
interpolates its spatial table (encoders.py:505-512), the auxiliary encoder is a plain length-T*N
VisionTransformer (:846-857) and the poolers take any token count (:859-885).  Here the auxiliary
encoder's GEMM rows are padded to the tile (vp_clip.cpp clip_video_chunk) and its attention takes a
partial last block of queries and keys (attention_long_kernel.h TAIL), or the sequence kernel at
T*N <= 256.

  * kernel: attention_long_bf16 at S = 300 / 520 / 1000 / 3136 vs the oracle, per element within
    2^-8 (|ref| + max|v|) (test_gpu_clip.py's bar for this kernel), at logit scales that take every
    numerator tier;
  * kernel: bf16 attention with key paddings beyond 256 keys (the forward's attention_masked), S = 300
    and 520, random paddings and a fully padded sequence, through vp_op_attention and
    vp_op_attention_masked (causal and not);
  * full-depth LvT-Base at 252 x 252, T = 16 (14 x 14 patches, 3136 auxiliary tokens) and 144 x 144,
    T = 3 (192), B = 1 and B = 3, fp32 and bf16, against the fp64 fixture g14 (tests/golden/make_golden.py):
    video, text, similarity and frame embeddings within 2e-5 (fp32); bf16 within 1e-3 (frames 2e-3, as
    test_gpu_lvt_large.py), the video bar widened to 1.1x a clip's bf16 cast floor where that floor (the
    distance of fp64 arithmetic on bf16-rounded parameters and frames, which fprop_dtype=bfloat16 mandates)
    is itself above 1e-3 (test_gpu_clip.py::test_clip_lvt_base_bf16_over_clips);
  * the temporal encoder beyond 256 frames (the generic attention over an interpolated table): T = 260
    with frame paddings at 144 x 144 and T = 300 at 36 x 36 (4 patches per frame), Base dims 1 + 1 layers,
    vs the fp64 oracle.

Parity unpinned by the reference (JAX absent): the bar is the oracle.
"""

import os

import numpy as np
import pytest
import torch

from oracle import videoprism_oracle as orc
from videoprism import _native as nat
from videoprism import encoders, models, params

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _qkv(num_seq, S, heads, seed, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    D = heads * 64
    q = torch.randn(num_seq * S, D, generator=g) * scale
    k = torch.randn(num_seq * S, D, generator=g) * scale
    v = torch.randn(num_seq * S, D, generator=g)
    return torch.cat([q, k, v], dim=1)


def _split(qkv, num_seq, S, heads):
    x = qkv.double().cpu().numpy().reshape(num_seq, S, 3, heads, 64)
    return [x[:, :, i].transpose(0, 2, 1, 3).reshape(num_seq * heads, S, 64) for i in range(3)]


def _merge(o, num_seq, S, heads):
    return o.reshape(num_seq, heads, S, 64).transpose(0, 2, 1, 3).reshape(num_seq * S, heads * 64)


# scale 0.1 keeps the logits in the linear tier, 0.3 / 1 in the polynomial ones, 3 in the exact form
@pytest.mark.parametrize("S,num_seq,heads,scale", [(300, 2, 12, 1.0), (520, 3, 4, 3.0), (1000, 1, 16, 0.1),
                                                   (3136, 1, 12, 0.3), (257, 2, 2, 1.0), (319, 1, 3, 2.0)])
def test_attention_long_bf16_partial_blocks(cuda, S, num_seq, heads, scale):
    qkv = _qkv(num_seq, S, heads, S + 3 * heads, scale).to(torch.bfloat16).to(cuda)
    # rows past the last sequence are poisoned: a load or a weight past S would show up
    buf = torch.full((num_seq * S + 512, 3 * heads * 64), float("nan"), dtype=torch.bfloat16, device=cuda)
    buf[:num_seq * S] = qkv
    out = torch.full((num_seq * S + 256, heads * 64), 7.0, dtype=torch.bfloat16, device=cuda)
    nat.op_attention(buf, num_seq, S, heads, 50.0, out=out)
    torch.cuda.synchronize()
    assert bool((out[num_seq * S:] == 7.0).all())  # no store past the last query
    q, k, v = _split(qkv, num_seq, S, heads)
    ref = _merge(orc.capped_softmax_attention(q, k, v, 50.0), num_seq, S, heads)
    err = np.abs(out[:num_seq * S].double().cpu().numpy() - ref)
    vmax = float(qkv[:, 2 * heads * 64:].float().abs().max())
    print(f"long attention S={S} (S % 256 = {S % 256}): max {err.max():.3e} mean {err.mean():.3e}")
    assert np.all(err <= 2 ** -8 * (np.abs(ref) + vmax)), err.max()


@pytest.mark.parametrize("op", ["attention", "masked", "masked_causal"])
@pytest.mark.parametrize("S,num_seq", [(300, 3), (520, 2)])
def test_attention_bf16_key_padding_beyond_256(cuda, op, S, num_seq):
    """bf16 attention with key paddings at S > 256 (T > 256 frames with frame_paddings, grids of more than
    256 patches with padded frames): random paddings, one half-padded and one fully padded sequence (uniform
    weights, as the reference's where(mask, logits, -0.7 FLT_MAX) + softmax, layers.py:51-89, 601-661)."""
    heads = 4
    qkv = _qkv(num_seq, S, heads, 5 * S + num_seq).to(torch.bfloat16).to(cuda)
    g = torch.Generator(device="cpu").manual_seed(S + 1)
    kp = (torch.rand(num_seq, S, generator=g) < 0.3).float()
    kp[0, S // 2:] = 1.0
    kp[-1] = 1.0
    kpd = kp.reshape(-1).to(cuda)
    causal = op == "masked_causal"
    if op == "attention":
        out = nat.op_attention(qkv, num_seq, S, heads, 50.0, key_pad=kpd)
    else:
        out = nat.op_attention_masked(qkv, num_seq, S, heads, 50.0, key_pad=kpd, causal=causal)
    torch.cuda.synchronize()
    q, k, v = _split(qkv, num_seq, S, heads)
    kpp = np.repeat(kp.numpy().reshape(num_seq, 1, S), heads, axis=1).reshape(-1, S)
    ref = _merge(orc.masked_attention(q, k, v, 50.0, kpp, causal), num_seq, S, heads)
    err = np.abs(out.double().cpu().numpy() - ref)
    vmax = float(qkv[:, 2 * heads * 64:].float().abs().max())
    print(f"{op} S={S}: max {err.max():.3e} mean {err.mean():.3e}")
    assert np.all(err <= 2 ** -8 * (np.abs(ref) + vmax)), err.max()


@pytest.fixture(scope="module")
def g14():
    g = np.load(os.path.join(GOLD, "g14_lvt_base_frame_sizes.npz"), allow_pickle=False)
    cfg = dict(models.CONFIGS[str(g["cfg"])])
    cfg["vocabulary_size"] = int(g["vocabulary_size"])
    var = params.synthetic_params(cfg, seed=int(g["param_seed"]), specs=params.clip_leaf_specs(cfg))
    return g, cfg, var


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("B", [1, 3])
@pytest.mark.parametrize("tag", ["s252_t16", "s144_t3"])
def test_lvt_base_frame_sizes_full_depth(cuda, g14, tag, B, bf16):
    g, cfg, var = g14
    size, T, vseed = (int(v) for v in g[f"{tag}/geometry"])
    video = np.random.default_rng(vseed).random((int(g["B"]), T, size, size, 3), dtype=np.float32)[:B]
    mdl = models.get_model("videoprism_lvt_public_v1_base", fprop_dtype=torch.bfloat16 if bf16 else None)
    mdl.vocabulary_size = cfg["vocabulary_size"]
    v, t, out = mdl.apply(var, video, g["text_token_ids"], g["text_paddings"], train=False,
                          return_intermediate=("frame_embeddings",))
    v, t = np.asarray(v, np.float64), np.asarray(t, np.float64)
    f = np.asarray(out["frame_embeddings"], np.float64)
    assert v.shape == (B, 768) and f.shape == (B, T, 768)
    ev = np.abs(v - g[f"{tag}/video_emb_f64"][:B]).max(axis=-1)
    et = np.abs(t - g[f"{tag}/text_emb_f64"]).max()
    es = np.abs(v @ t.T - g[f"{tag}/similarity_f64"][:B]).max()
    ef = np.abs(f - g[f"{tag}/frame_emb_f64"][:B]).max()
    floor = np.abs(g[f"{tag}/cast_floor_emb"][:B] - g[f"{tag}/video_emb_f64"][:B]).max(axis=-1)
    fmt = lambda a: "[" + " ".join(f"{v:.3e}" for v in a) + "]"  # noqa: E731
    print(f"LvT-B {tag} B={B} {'bf16' if bf16 else 'f32'}: video {fmt(ev)} (cast floor {fmt(floor)}) text {et:.3e} "
          f"similarity {es:.3e} frames {ef:.3e}")
    if bf16:
        vbar = np.maximum(1e-3, 1.1 * floor)
        assert np.all(ev <= vbar) and et <= 1e-3 and es <= 1e-3 and ef <= 2e-3, (ev, floor, et, es, ef)
    else:
        assert ev.max() <= 2e-5 and et <= 2e-5 and es <= 2e-5 and ef <= 2e-5, (ev, et, es, ef)


def _small_cfg():
    cfg = dict(models.CONFIGS["videoprism_v1_base"])
    cfg.update(num_spatial_layers=1, num_temporal_layers=1)
    return cfg


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("T,size,padded", [(260, 144, True), (300, 36, False)])
def test_temporal_beyond_256_frames(cuda, bf16, T, size, padded):
    """The temporal encoder at T > 256 (vp_prepare_frames' 16 -> T table, the generic attention over T keys),
    with the last frames of clip 1 padded (T = 260, encoders.py:440-447) or without paddings at 4 patches per
    frame (T = 300)."""
    cfg = _small_cfg()
    var = params.synthetic_params(cfg, seed=T)
    video = np.random.default_rng(T + 1).random((2, T, size, size, 3), dtype=np.float32)
    fp = None
    if padded:
        fp = np.zeros((2, T), np.float32)
        fp[1, T - 37:] = 1.0
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedEncoder(**cfg),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    emb, _ = m.apply(var, video, frame_paddings=fp)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, "f64", frame_paddings=fp)
    emb = np.asarray(emb, np.float64)
    if bf16:
        perr = np.abs(orc.l2_normalize(emb.mean(1)) - orc.l2_normalize(ref.mean(1))).max()
        mean_err = np.abs(emb - ref).mean()
        print(f"T={T} {size}x{size} padded={padded} bf16: pooled {perr:.3e} token mean-abs {mean_err:.3e}")
        assert perr <= 1e-3 and mean_err <= 2e-2
    else:
        err = np.abs(emb - ref).max()
        print(f"T={T} {size}x{size} padded={padded} f32: max-abs {err:.3e}")
        assert err <= 1e-5


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("size,T", [(36, 3), (108, 5), (90, 12)])
def test_lvt_reduced_depth_small_grids(cuda, size, T, bf16):
    """LvT-Base dims, 1 + 1 vision / 1 auxiliary / 1 text layer, at grids of 2x2 (12 auxiliary tokens: the
    temporal kernel), 6x6 (180: the sequence kernel) and 5x5 at T = 12 (300: the long kernel's partial
    block), B = 2, vs the fp64 oracle on the fly."""
    cfg = dict(models.CONFIGS["videoprism_lvt_v1_base"], vocabulary_size=100, num_spatial_layers=1,
               num_temporal_layers=1, num_auxiliary_layers=1, num_unimodal_layers=1)
    var = params.synthetic_params(cfg, size + T, specs=params.clip_leaf_specs(cfg))
    video = np.random.default_rng(size).random((2, T, size, size, 3), dtype=np.float32)
    ids = np.random.default_rng(T).integers(0, 100, (2, 9)).astype(np.int32)
    pads = np.zeros((2, 9), np.float32)
    pads[1, 4:] = 1.0
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**cfg),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    v, t, out = m.apply(var, video, ids, pads, return_intermediate=("frame_embeddings",))
    rv, rt, rout = orc.video_clip(var["params"], cfg, video, ids, pads, "f64", return_intermediate=("frame_embeddings",))
    ev, et = np.abs(v - rv).max(), np.abs(t - rt).max()
    ef = np.abs(out["frame_embeddings"] - rout["frame_embeddings"]).max()
    print(f"LvT-B 1+1/1/1 {size}x{size} T={T} ({T * (size // 18) ** 2} aux tokens) {'bf16' if bf16 else 'f32'}: "
          f"video {ev:.3e} frames {ef:.3e} text {et:.3e}")
    tol = 2e-3 if bf16 else 2e-5
    assert ev <= tol and ef <= tol and et <= tol, (ev, ef, et)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bf16", [False, True])
def test_lvt_large_dims_252_uint8_padded(cuda, bf16):
    """LvT-Large dims (D 1024, 16 heads), 1 + 1 vision / 2 auxiliary / 1 text layer, 252 x 252 uint8 frames (the
    /255 ingest), T = 7 with the last two frames of clip 1 padded (the vision encoder masks them; the auxiliary
    encoder and the poolers see no paddings, encoders.py:846-885): 1372 auxiliary tokens (partial last block)."""
    cfg = dict(models.CONFIGS["videoprism_lvt_v1_large"], vocabulary_size=100, num_spatial_layers=1,
               num_temporal_layers=1, num_auxiliary_layers=2, num_unimodal_layers=1)
    var = params.synthetic_params(cfg, 31, specs=params.clip_leaf_specs(cfg))
    frames = np.random.default_rng(31).integers(0, 256, (2, 7, 252, 252, 3), dtype=np.uint8)
    fp = np.zeros((2, 7), np.float32)
    fp[1, 5:] = 1.0
    ids = np.random.default_rng(32).integers(0, 100, (3, 12)).astype(np.int32)
    pads = np.zeros((3, 12), np.float32)
    pads[2, 6:] = 1.0
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**cfg),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    v, t, out = m.apply(var, frames, ids, pads, frame_paddings=fp, return_intermediate=("frame_embeddings",))
    video = frames.astype(np.float32) / np.float32(255.0)  # video_utils.py:94
    rv, rt, rout = orc.video_clip(var["params"], cfg, video, ids, pads, "f64",
                                  return_intermediate=("frame_embeddings",), frame_paddings=fp)
    ev, et = np.abs(v - rv).max(), np.abs(t - rt).max()
    ef = np.abs(out["frame_embeddings"] - rout["frame_embeddings"]).max()
    print(f"LvT-L dims 252x252 uint8 T=7 padded {'bf16' if bf16 else 'f32'}: video {ev:.3e} frames {ef:.3e} text {et:.3e}")
    tol = 2e-3 if bf16 else 2e-5
    assert ev <= tol and ef <= tol and et <= tol, (ev, ef, et)
