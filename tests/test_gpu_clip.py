"""MI355X parity of the LvT video-text path against the NumPy oracle,
through the C-ABI (vp_clip_*, vp_op_attention*, vp_op_similarity).

Tolerances (written here; measured values are printed and recorded in DESIGN.md):
  * long-sequence bf16 attention (auxiliary encoder, S = T*N): per element
    2^-8 (|ref| + max|v|) -- bf16 rounding of the numerators and of the output;
  * masked fp32-math attention (text tower): 3e-5 (fp32), 2^-8 (|ref| + max|v|) (bf16 I/O);
  * end-to-end L2-normalised video / frame / text embeddings vs oracle fp64: 2e-5 (fprop
    float32) and 1e-3 (fprop bfloat16, the north_star bar).
"""

import os

import numpy as np
import pytest
import torch

from oracle import videoprism_oracle as orc
from videoprism import _native as nat
from videoprism import encoders, models, params

pytestmark = pytest.mark.gpu


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


# scale 0.125 keeps every logit below 0.48*cap (one-transcendental polynomial numerator), the
# larger scales put logits past it in most tiles (exact three-transcendental path)
@pytest.mark.parametrize("S,num_seq,heads,scale", [(512, 2, 12, 1.0), (1024, 1, 3, 3.0),
                                                   (4096, 1, 2, 1.0), (768, 3, 16, 2.0),
                                                   (512, 2, 12, 0.125), (2048, 1, 4, 0.3)])
def test_attention_long_bf16(cuda, S, num_seq, heads, scale):
    qkv = _qkv(num_seq, S, heads, S + heads, scale).to(torch.bfloat16).to(cuda)
    out = nat.op_attention(qkv, num_seq, S, heads, 50.0)
    torch.cuda.synchronize()
    q, k, v = _split(qkv, num_seq, S, heads)
    ref = _merge(orc.capped_softmax_attention(q, k, v, 50.0), num_seq, S, heads)
    err = np.abs(out.double().cpu().numpy() - ref)
    vmax = float(qkv[:, 2 * heads * 64:].float().abs().max())
    print(f"long attention S={S}: max {err.max():.3e} mean {err.mean():.3e}")
    assert np.all(err <= 2 ** -8 * (np.abs(ref) + vmax)), err.max()


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("S,num_seq,causal", [(65, 4, True), (65, 3, False), (130, 2, True), (7, 5, True),
                                             (33, 9, True), (256, 2, True), (300, 2, True)])
def test_attention_masked(cuda, bf16, S, num_seq, causal):
    """Causal + key-padding merge (layers.py:111-179): bf16 16 < S <= 256 runs on the MFMA sequence kernel (the
    text tower's path), S <= 16, S > 256 and fp32 on the generic kernel."""
    heads = 12
    qkv = _qkv(num_seq, S, heads, S * 7 + num_seq)
    if bf16:
        qkv = qkv.to(torch.bfloat16)
    qkv = qkv.to(cuda)
    g = torch.Generator(device="cpu").manual_seed(S)
    kp = (torch.rand(num_seq, S, generator=g) < 0.3).float()
    kp[0, S // 2:] = 1.0       # the reference test's half-padded text (models_test.py:61-69)
    kp[-1] = 1.0               # fully padded sequence -> uniform rows
    out = nat.op_attention_masked(qkv, num_seq, S, heads, 50.0, key_pad=kp.reshape(-1).to(cuda),
                                  causal=causal)
    torch.cuda.synchronize()
    q, k, v = _split(qkv, num_seq, S, heads)
    kpp = np.repeat(kp.numpy().reshape(num_seq, 1, S), heads, axis=1).reshape(-1, S)
    ref = _merge(orc.masked_attention(q, k, v, 50.0, kpp, causal), num_seq, S, heads)
    err = np.abs(out.double().cpu().numpy() - ref)
    if bf16:
        vmax = float(qkv[:, 2 * heads * 64:].float().abs().max())
        assert np.all(err <= 2 ** -8 * (np.abs(ref) + vmax)), err.max()
    else:
        assert err.max() < 3e-5, err.max()


def test_similarity(cuda):
    g = torch.Generator(device="cpu").manual_seed(0)
    a = torch.randn(5, 768, generator=g)
    b = torch.randn(3, 768, generator=g)
    out = nat.op_similarity(a.to(cuda), b.to(cuda))
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy(), (a.double() @ b.double().T).numpy(), rtol=1e-5, atol=1e-4)


def _lvt_cfg(name="videoprism_lvt_v1_base", **kw):
    c = dict(models.CONFIGS[name])
    c["vocabulary_size"] = 1000
    c.update(kw)
    return c


def _text(Q, L, seed, V):
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, V, (Q, L)).astype(np.int32)
    pads = np.zeros((Q, L), np.float32)
    pads[0, L // 2:] = 1.0           # models_test.py:61-69: second half padded
    if Q > 2:
        pads[2, 3:] = 1.0
    return ids, pads


def _run_clip(cfg, bf16, B, T, Q, L, seed):
    var = params.synthetic_params(cfg, seed, specs=params.clip_leaf_specs(cfg))
    video = np.random.default_rng(seed).random((B, T, 288, 288, 3), dtype=np.float32)
    ids, pads = _text(Q, L, seed, cfg["vocabulary_size"])
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**cfg),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    eng = m.engine(var, torch.cuda.current_device())
    x = torch.from_numpy(video).cuda()
    if bf16:
        x = x.to(torch.bfloat16)
    vemb, femb, _, st = eng.encode_video(x, want_frames=True, want_spatiotemporal=True)
    temb = eng.encode_text(torch.from_numpy(ids).cuda(), torch.from_numpy(pads).cuda())
    torch.cuda.synchronize()
    rv, rt, out = orc.video_clip(var["params"], cfg, video, ids, pads, "f64",
                                 return_intermediate=("frame_embeddings", "spatiotemporal_features"))
    return (vemb.cpu().numpy(), femb.cpu().numpy(), temb.cpu().numpy(), st.float().cpu().numpy(),
            rv, out["frame_embeddings"], rt, out["spatiotemporal_features"])


@pytest.mark.parametrize("bf16", [False, True])
def test_clip_reduced_depth(cuda, bf16):
    """LvT-Base dims (D 768, 12 heads, pooler dh 256) with 1+1 vision, 2 auxiliary and 2 text
    layers; B=2, T=2 (auxiliary attention over 512 tokens), Q=3 texts of 16 tokens."""
    cfg = _lvt_cfg(num_spatial_layers=1, num_temporal_layers=1, num_unimodal_layers=2)
    v, f, t, st, rv, rf, rt, rst = _run_clip(cfg, bf16, 2, 2, 3, 16, 7)
    ev, ef, et = np.abs(v - rv).max(), np.abs(f - rf).max(), np.abs(t - rt).max()
    print(f"clip {'bf16' if bf16 else 'f32'}: video {ev:.3e} frames {ef:.3e} text {et:.3e} "
          f"spatiotemporal mean {np.abs(st - rst).mean():.3e}")
    tol = 1e-3 if bf16 else 2e-5
    assert ev <= tol and ef <= tol and et <= tol, (ev, ef, et)
    np.testing.assert_allclose(np.linalg.norm(v, axis=-1), 1.0, rtol=1e-5)


def test_clip_full_lvt_base_bf16(cuda):
    """Full LvT-Base depth (12+4 vision, 2 auxiliary, 12 text layers), B=1, T=8 (auxiliary
    attention over 2048 tokens), two 64-token texts (second half of one padded)."""
    cfg = _lvt_cfg()
    v, f, t, _, rv, rf, rt, _ = _run_clip(cfg, True, 1, 8, 2, 64, 11)
    ev, ef, et = np.abs(v - rv).max(), np.abs(f - rf).max(), np.abs(t - rt).max()
    print(f"full LvT-B bf16: video {ev:.3e} frames {ef:.3e} text {et:.3e}")
    assert ev <= 1e-3 and ef <= 2e-3 and et <= 1e-3, (ev, ef, et)


@pytest.mark.timeout(300)
def test_clip_lvt_base_bf16_over_clips(cuda):
    """Full-depth LvT-Base bf16 over 8 clips (fixture g13: seeds 11..18, the construction of
    test_clip_full_lvt_base_bf16).  At one clip that test's 1e-3 bar sits at the bf16 noise floor: casting
    the parameters and frames alone (fprop_dtype=bfloat16 mandates it) moves these clips' video embeddings
    8.0e-4 .. 1.01e-3 from fp64.  This gate asks that the kernels add no error beyond that cast: the mean
    over the clips within the cast floor's mean, and every clip within 1.1x the largest cast floor."""
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "g13_lvt_base_clips.npz"),
                allow_pickle=False)
    cfg = _lvt_cfg()
    cfg["vocabulary_size"] = int(g["vocabulary_size"])
    errs, floors = [], []
    for i, seed in enumerate(g["seeds"]):
        var = params.synthetic_params(cfg, int(seed), specs=params.clip_leaf_specs(cfg))
        video = np.random.default_rng(int(seed)).random((1, int(g["T"]), 288, 288, 3), dtype=np.float32)
        m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**cfg), fprop_dtype=torch.bfloat16)
        v = m.engine(var, torch.cuda.current_device()).encode_video(torch.from_numpy(video).cuda().to(torch.bfloat16))[0]
        torch.cuda.synchronize()
        ref = g["video_emb_f64"][i]
        errs.append(float(np.abs(v.cpu().numpy().astype(np.float64)[0] - ref).max()))
        floors.append(float(np.abs(g["cast_floor_emb"][i] - ref).max()))
        del m
    errs, floors = np.array(errs), np.array(floors)
    print(f"LvT-B bf16 over {len(errs)} clips: video max-abs mean {errs.mean():.3e} max {errs.max():.3e}; "
          f"cast floor mean {floors.mean():.3e} max {floors.max():.3e}")
    assert errs.mean() <= floors.mean() and errs.max() <= 1.1 * floors.max(), (errs, floors)


def test_clip_apply_api(cuda):
    """The drop-in call: get_model(lvt).apply(variables, inputs, ids, paddings) -> numpy."""
    cfg = _lvt_cfg(num_spatial_layers=1, num_temporal_layers=1, num_auxiliary_layers=1,
                   num_unimodal_layers=1)
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**cfg))
    var = m.init(3)
    video = np.random.default_rng(1).random((1, 2, 288, 288, 3), dtype=np.float32)
    ids, pads = _text(2, 8, 1, cfg["vocabulary_size"])
    v, t, out = m.apply(var, video, ids, pads, return_intermediate=True)
    assert v.shape == (1, 768) and t.shape == (2, 768)
    assert set(out) == {"frame_embeddings", "spatial_features", "spatiotemporal_features"}
    v2, t2, out2 = m.apply(var, video)
    assert t2 is None and out2 == {}
    np.testing.assert_allclose(v, v2, atol=1e-6)
    rv, rt, _ = orc.video_clip(var["params"], cfg, video, ids, pads, "f64")
    assert np.abs(v - rv).max() < 2e-5 and np.abs(t - rt).max() < 2e-5


@pytest.mark.parametrize("bf16", [False, True])
def test_clip_large_dims_padded_frames(cuda, bf16):
    """LvT-Large dims (D 1024, 16 heads: pooler dh 256 with 2H = 32 logit columns, temporal
    pos-emb 8 -> T), reduced depth; a padded frame in the vision encoder (the auxiliary
    encoder and the pooler see no paddings, encoders.py:846-872); out-of-range text ids clamp."""
    cfg = _lvt_cfg("videoprism_lvt_v1_large", num_spatial_layers=1, num_temporal_layers=1,
                   num_auxiliary_layers=1, num_unimodal_layers=1)
    var = params.synthetic_params(cfg, 21, specs=params.clip_leaf_specs(cfg))
    video = np.random.default_rng(21).random((2, 2, 288, 288, 3), dtype=np.float32)
    fpad = np.zeros((2, 2), np.float32)
    fpad[1, 1] = 1.0
    ids, pads = _text(3, 12, 21, cfg["vocabulary_size"])
    ids[0, 0] = cfg["vocabulary_size"] + 5   # clamps to V-1, as a JAX gather does
    ids[1, 1] = -3                           # clamps to 0
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**cfg),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    v, t, out = m.apply(var, video, ids, pads, frame_paddings=fpad,
                        return_intermediate=("frame_embeddings",))
    rv, rt, rout = orc.video_clip(var["params"], cfg, video, ids, pads, "f64",
                                  return_intermediate=("frame_embeddings",), frame_paddings=fpad)
    ev, et = np.abs(v - rv).max(), np.abs(t - rt).max()
    ef = np.abs(out["frame_embeddings"] - rout["frame_embeddings"]).max()
    print(f"LvT-L dims {'bf16' if bf16 else 'f32'}: video {ev:.3e} frames {ef:.3e} text {et:.3e}")
    tol = 2e-3 if bf16 else 2e-5   # bf16 outputs are returned in bf16 (2^-9 relative)
    assert ev <= tol and ef <= tol and et <= tol, (ev, ef, et)
