"""End-to-end parity of the MI355X FactorizedEncoder forward (through the C-ABI, via the
drop-in `models.get_model(...).apply`) against the NumPy oracle.

Tolerances (written here, measured on MI355X):
  * fprop float32 vs oracle fp64: max-abs <= 1e-5 on LayerNorm-ed O(1) outputs (the north_star
    bar; the measured value is printed).
  * fprop bfloat16 vs oracle fp64: bf16 rounding of every GEMM operand makes per-token
    deviations of a few 1e-2 unavoidable; we bound mean-abs <= 2e-2,
    and max-abs of the L2-normalised mean-pooled clip embedding <= 1e-3 (north_star).
"""

import numpy as np
import pytest
import torch

from oracle import videoprism_oracle as orc
from videoprism import models, params

pytestmark = pytest.mark.gpu


def _cfg(base, **kw):
    c = dict(models.CONFIGS[base])
    c.update(kw)
    return c


def _model(cfg, bf16):
    m = models.get_model(None, model_fn=lambda: models.encoders.FactorizedEncoder(**cfg),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    return m


def _video(B, T, H, seed, dist="uniform"):
    rng = np.random.default_rng(seed)
    if dist == "uniform":
        return rng.random((B, T, H, H, 3), dtype=np.float32)
    return rng.normal(0.0, 0.1, (B, T, H, H, 3)).astype(np.float32)


def _pool_l2(e):
    m = e.astype(np.float64).mean(axis=1)
    return m / np.sqrt((m * m).sum(-1, keepdims=True) + 1e-12)


def _run(cfg, variables, video, bf16, **kw):
    mdl = _model(cfg, bf16)
    return mdl.apply(variables, video, train=False, **kw)


REDUCED_BASE = _cfg("videoprism_v1_base", num_spatial_layers=2, num_temporal_layers=1)
REDUCED_LARGE = _cfg("videoprism_v1_large", num_spatial_layers=2, num_temporal_layers=1)


@pytest.mark.parametrize("dist", ["uniform", "normal"])
def test_base_dims_f32(cuda, dist):
    cfg = REDUCED_BASE
    var = params.synthetic_params(cfg, seed=1)
    video = _video(1, 2, 288, 3, dist)
    emb, _ = _run(cfg, var, video, bf16=False)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, mode="f64")
    err = np.abs(emb - ref)
    print(f"f32 base-dims max-abs {err.max():.3e} mean-abs {err.mean():.3e}")
    assert emb.shape == (1, 2 * 256, 768)
    assert err.max() <= 1e-5


def test_base_dims_bf16(cuda):
    cfg = REDUCED_BASE
    var = params.synthetic_params(cfg, seed=1)
    video = _video(2, 2, 288, 4)
    emb, _ = _run(cfg, var, video, bf16=True)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, mode="f64")
    err = np.abs(emb - ref)
    perr = np.abs(_pool_l2(emb) - _pool_l2(ref))
    print(f"bf16 base-dims token max-abs {err.max():.3e} mean-abs {err.mean():.3e}; "
          f"pooled-l2 max-abs {perr.max():.3e}")
    assert err.mean() <= 2e-2
    assert perr.max() <= 1e-3


def test_frame_paddings_and_intermediate_f32(cuda):
    cfg = REDUCED_BASE
    var = params.synthetic_params(cfg, seed=2)
    video = _video(2, 4, 288, 5)
    fp = np.zeros((2, 4), np.float32)
    fp[:, 2:] = 1.0          # encoders_test.py:138-142 half-padded frames
    fp[1, :] = 1.0           # a fully padded clip: uniform attention everywhere
    emb, out = _run(cfg, var, video, bf16=False, frame_paddings=fp,
                    return_intermediate=True)
    ref, rout = orc.factorized_encoder(var["params"], video, cfg, mode="f64",
                                       frame_paddings=fp, return_intermediate=True)
    assert set(out) == {"spatial_features"}
    e1, e2 = np.abs(emb - ref).max(), np.abs(out["spatial_features"] - rout["spatial_features"]).max()
    print(f"f32 padded frames: embeddings max-abs {e1:.3e}, spatial_features {e2:.3e}")
    assert e1 <= 1e-5 and e2 <= 1e-5


def test_frame_paddings_bf16(cuda):
    cfg = REDUCED_BASE
    var = params.synthetic_params(cfg, seed=2)
    video = _video(2, 4, 288, 6)
    fp = np.zeros((2, 4), np.float32)
    fp[0, 1] = 1.0
    fp[1, 3] = 1.0
    emb, _ = _run(cfg, var, video, bf16=True, frame_paddings=fp)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, mode="f64", frame_paddings=fp)
    assert np.abs(emb - ref).mean() <= 2e-2


def test_large_dims_temporal_interpolation_f32(cuda):
    """Large: pos_emb T=8 interpolated to 16 input frames (encoders.py:551-552)."""
    cfg = REDUCED_LARGE
    var = params.synthetic_params(cfg, seed=3)
    video = _video(1, 16, 288, 7)
    emb, _ = _run(cfg, var, video, bf16=False)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, mode="f64")
    assert emb.shape == (1, 16 * 256, 1024)
    err = np.abs(emb - ref).max()
    print(f"f32 large dims T 8->16: max-abs {err:.3e}")
    assert err <= 1e-5


def test_batch_invariance_bitwise_bf16(cuda):
    """Size-independent property: each clip's output is bitwise independent of the
    batch it was run in (every kernel reduces in a batch-independent order)."""
    cfg = REDUCED_BASE
    var = params.synthetic_params(cfg, seed=4)
    video = torch.from_numpy(_video(4, 4, 288, 8)).to(cuda).to(torch.bfloat16)
    mdl = _model(cfg, True)
    full, _ = mdl.apply(var, video)
    for b in range(4):
        one, _ = mdl.apply(var, video[b:b + 1].contiguous())
        assert torch.equal(one[0], full[b])


def test_full_base_b1_f32_vs_oracle(cuda):
    """Full videoprism_public_v1_base, B=1, T=8 (models_test.py:36-53 shape pin)."""
    cfg = models.CONFIGS["videoprism_v1_base"]
    var = params.synthetic_params(cfg, seed=0)
    video = _video(1, 8, 288, 9, "normal")
    mdl = models.get_model("videoprism_public_v1_base")
    emb, _ = mdl.apply(var, video, train=False)
    assert emb.shape == (1, 8 * 16 ** 2, 768)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, mode="f32")
    err = np.abs(emb - ref)
    print(f"full base f32 vs oracle-f32 max-abs {err.max():.3e} mean-abs {err.mean():.3e}")
    assert err.max() <= 1e-5


def test_full_base_b1_bf16_vs_oracle(cuda):
    """Full-depth videoprism_public_v1_base in bf16 (bf16 residual stream, as Flax with
    fprop_dtype=bfloat16): the north_star bound is on the L2-normalised mean-pooled clip
    embedding, max-abs <= 1e-3 vs the fp64 oracle; token errors are printed against both the
    fp64 oracle and the oracle's bf16 emulation of the reference."""
    cfg = models.CONFIGS["videoprism_v1_base"]
    var = params.synthetic_params(cfg, seed=0)
    video = _video(1, 8, 288, 9, "normal")
    mdl = models.get_model("videoprism_public_v1_base", fprop_dtype=torch.bfloat16)
    emb, _ = mdl.apply(var, video, train=False)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, mode="f64")
    emu, _ = orc.factorized_encoder(var["params"], video, cfg, mode="bf16")
    err, err_emu = np.abs(emb - ref), np.abs(emb - emu)
    perr = np.abs(_pool_l2(emb) - _pool_l2(ref))
    print(f"full base bf16: vs f64 token mean-abs {err.mean():.3e} max {err.max():.3e}; vs bf16-emulation "
          f"mean-abs {err_emu.mean():.3e}; reference-emulation vs f64 mean-abs {np.abs(emu - ref).mean():.3e}; "
          f"pooled-l2 max-abs {perr.max():.3e}")
    assert perr.max() <= 1e-3
    assert err.mean() <= 3e-2


@pytest.mark.parametrize("base", ["videoprism_v1_base", "videoprism_v1_large"])
def test_temporal_attention_fused_vs_unfused_and_oracle(cuda, base):
    """bf16 at T = 16 runs the temporal layers' attention inside the q|k|v projection
    (EPI_QK_TATTN_LN + EPI_V_TATTN_LN); all-zero frame paddings take the unfused path (GEMM ->
    attn_temporal_kernel) on the same inputs.  Both against the fp64 oracle (2+2 layers, B = 2,
    clips 2 x 16 x 288 x 288): token mean-abs and pooled max-abs bars as above, and fused vs
    unfused within bf16 rounding of the probabilities (the fused path rounds the normalised
    probabilities, the unfused one the numerators)."""
    cfg = _cfg(base, num_spatial_layers=2, num_temporal_layers=2)
    var = params.synthetic_params(cfg, seed=31)
    video = _video(2, 16, 288, 32)
    fused, _ = _run(cfg, var, video, bf16=True)
    unfused, _ = _run(cfg, var, video, bf16=True, frame_paddings=np.zeros((2, 16), np.float32))
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, mode="f64")
    for tag, e in (("fused", fused), ("unfused", unfused)):
        err = np.abs(e - ref)
        perr = np.abs(_pool_l2(e) - _pool_l2(ref)).max()
        print(f"{base} T=16 {tag}: token max-abs {err.max():.3e} mean-abs {err.mean():.3e}; pooled {perr:.3e}")
        assert err.mean() <= 2e-2 and perr <= 1e-3
    d = np.abs(fused - unfused)
    print(f"fused vs unfused: max-abs {d.max():.3e} mean-abs {d.mean():.3e}")
    assert d.mean() <= 5e-3
