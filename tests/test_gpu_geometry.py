"""Frame sizes other than 288x288 and clip lengths beyond 16: the spatial
positional table is interpolated like encoders.py:497-512 (jax.image.resize 'bilinear',
antialiased when shrinking; vp_prepare_geometry), GEMM rows are padded to the tile, and the
attention falls back to the generic fp32-math kernel for S != 256 / T > 16.  Checked against the
oracle fp64 (whose resize is pinned by the torch restatement and MLX's upsampling, test_oracle.py).
Tolerances as in test_gpu_encoder.py: fp32 max-abs 1e-5; bf16 token mean-abs 2e-2 and
L2-normalised mean-pooled embedding max-abs 1e-3."""

import numpy as np
import pytest
import torch

from oracle import videoprism_oracle as orc
from videoprism import encoders, models, params

pytestmark = pytest.mark.gpu


def _run(H, T, bf16, seed=0, B=1):
    cfg = dict(models.CONFIGS["videoprism_v1_base"])
    cfg.update(num_spatial_layers=1, num_temporal_layers=1)
    var = params.synthetic_params(cfg, seed=seed)
    video = np.random.default_rng(seed).random((B, T, H, H, 3), dtype=np.float32)
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedEncoder(**cfg),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    emb, _ = m.apply(var, video)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, "f64")
    return np.asarray(emb, np.float64), ref


def _pooled(x):
    return orc.l2_normalize(x.mean(axis=1))


@pytest.mark.parametrize("H,T", [(144, 3), (360, 2), (216, 20)])
def test_geometry_f32(cuda, H, T):
    emb, ref = _run(H, T, False)
    assert emb.shape == ref.shape == (1, T * (H // 18) ** 2, 768)
    err = np.abs(emb - ref).max()
    print(f"f32 H={H} T={T}: max-abs {err:.3e}")
    assert err < 1e-5


@pytest.mark.parametrize("H,T", [(144, 3), (360, 2), (288, 20)])
def test_geometry_bf16(cuda, H, T):
    emb, ref = _run(H, T, True, seed=1)
    mean_err = np.abs(emb - ref).mean()
    pool_err = np.abs(_pooled(emb) - _pooled(ref)).max()
    print(f"bf16 H={H} T={T}: token mean-abs {mean_err:.3e} pooled {pool_err:.3e}")
    assert mean_err < 2e-2 and pool_err < 1e-3
