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


@pytest.mark.parametrize("P", [16, 9])
def test_other_patch_sizes_bf16(cuda, P):
    """Patch sizes other than 18 on the 16 x 16 grid (H = 16 P): even P takes the fused patch
    embedding straight from the frames, odd P (16-B chunks only 2-B aligned) patchify + GEMM
    (vp_kernels.h video_patch_ok).  Base dims, 1+1 layers, vs the oracle fp64."""
    cfg = dict(models.CONFIGS["videoprism_v1_base"])
    cfg.update(num_spatial_layers=1, num_temporal_layers=1, patch_size=P)
    var = params.synthetic_params(cfg, seed=P)
    video = np.random.default_rng(P).random((2, 4, 16 * P, 16 * P, 3), dtype=np.float32)
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedEncoder(**cfg), fprop_dtype=torch.bfloat16)
    emb, _ = m.apply(var, video)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, "f64")
    emb = np.asarray(emb, np.float64)
    mean_err = np.abs(emb - ref).mean()
    pool_err = np.abs(_pooled(emb) - _pooled(ref)).max()
    print(f"bf16 P={P}: token mean-abs {mean_err:.3e} pooled {pool_err:.3e}")
    assert mean_err < 2e-2 and pool_err < 1e-3


def test_misaligned_frames_take_the_patchify_path(cuda):
    """Frames at an address the fused path's chunk reads (4 B) or video_to_bf16's vector loads
    (16 B for fp32, 4 B for uint8) do not meet -- a view into a larger buffer, handed to the engine
    as it is (apply() would cast fp32 frames to a fresh, aligned bf16 tensor) -- run patchify +
    GEMM: bf16 / fp32 / uint8 views at odd offsets give bitwise the same result as each other
    (the fp32 values are IEEE u8 / 255, the kernel's own conversion), within the pooled bar of
    the oracle and within bf16 rounding of the aligned (fused) forward."""
    cfg = dict(models.CONFIGS["videoprism_v1_base"])
    cfg.update(num_spatial_layers=1, num_temporal_layers=1)
    var = params.synthetic_params(cfg, seed=31)
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedEncoder(**cfg), fprop_dtype=torch.bfloat16)
    eng = m.engine(var, torch.cuda.current_device())
    shape = (1, 2, 288, 288, 3)
    n = int(np.prod(shape))
    u8n = np.random.default_rng(31).integers(0, 256, n, dtype=np.uint8)
    f32n = u8n.astype(np.float32) / np.float32(255.0)
    u8 = torch.from_numpy(u8n).to(cuda)
    f32 = torch.from_numpy(f32n).to(cuda)
    bf = f32.to(torch.bfloat16)
    outs = {}
    for name, flat in (("bf16", bf), ("f32", f32), ("u8", u8)):
        buf = torch.zeros(n + 1, dtype=flat.dtype, device=cuda)
        buf[1:] = flat
        view = buf[1:].view(shape)
        assert view.is_contiguous() and view.data_ptr() % (16 if flat.dtype == torch.float32 else 4) != 0
        outs[name] = eng.forward(view)[0].clone()
    aligned = eng.forward(bf.view(shape).contiguous())[0]
    torch.cuda.synchronize()
    assert torch.equal(outs["bf16"], outs["f32"]) and torch.equal(outs["bf16"], outs["u8"])
    ref, _ = orc.factorized_encoder(var["params"], f32n.reshape(shape), cfg, "f64")
    got = outs["bf16"].double().cpu().numpy()
    fused = aligned.double().cpu().numpy()
    pool_err = np.abs(_pooled(got) - _pooled(ref)).max()
    mean_err, mean_fused = np.abs(got - ref).mean(), np.abs(fused - ref).mean()
    print(f"misaligned frames: pooled {pool_err:.3e} vs oracle; token mean-abs {mean_err:.3e} (aligned, fused "
          f"patch embedding: {mean_fused:.3e})")
    # the two patch embeddings differ only in their fp32 summation order (test_gpu_kernels.py
    # test_patch_embed_fused_from_frames): both forwards are equally close to fp64
    assert pool_err < 1e-3
    assert mean_err <= 1.1 * mean_fused
