"""uint8 frame ingest: frames as uint8 [0, 255] are normalised on device in
the patchify kernel exactly as the reference's loader does (video_utils.py:94,
float32(v) / 255.0), so the result is bitwise the one of the float path fed with v / 255."""

import numpy as np
import pytest
import torch

from oracle import videoprism_oracle as orc
from videoprism import _native as nat
from videoprism import encoders, models, params

pytestmark = pytest.mark.gpu


def _frames(B, T, seed):
    return np.random.default_rng(seed).integers(0, 256, (B, T, 288, 288, 3), dtype=np.uint8)


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_patchify_u8(cuda, out_dtype):
    v = _frames(1, 2, 0).reshape(2, 288, 288, 3)
    got = nat.op_patchify(torch.from_numpy(v).to(cuda), 18, 1024, out_dtype=out_dtype)
    torch.cuda.synchronize()
    ref = orc.image_to_patch(v.astype(np.float32) / np.float32(255.0), 18).reshape(-1, 972)
    ref = torch.from_numpy(np.pad(ref, ((0, 0), (0, 52)))).to(out_dtype)
    assert torch.equal(got.cpu(), ref)


@pytest.mark.parametrize("bf16", [False, True])
def test_apply_u8_bitwise_equals_normalised_float(cuda, bf16):
    cfg = dict(models.CONFIGS["videoprism_v1_base"])
    cfg.update(num_spatial_layers=1, num_temporal_layers=1)
    var = params.synthetic_params(cfg, seed=2)
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedEncoder(**cfg),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    v = _frames(1, 2, 1)
    e8, _ = m.apply(var, v)
    ef, _ = m.apply(var, v.astype(np.float32) / np.float32(255.0))
    np.testing.assert_array_equal(e8, ef)


def test_apply_three_input_dtypes_bitwise_bf16(cuda):
    """bf16 forward on the 16 x 16 patch grid: the patch embedding reads bf16 frames directly
    (gemm_bf16_w4_video); f32 and uint8 frames are converted to bf16 frames first with the patchify
    kernels' per-value conversion.  All three input dtypes give bitwise the same embedding."""
    cfg = dict(models.CONFIGS["videoprism_v1_base"])
    cfg.update(num_spatial_layers=1, num_temporal_layers=1)
    var = params.synthetic_params(cfg, seed=3)
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedEncoder(**cfg), fprop_dtype=torch.bfloat16)
    v8 = _frames(2, 2, 4)
    vf = v8.astype(np.float32) / np.float32(255.0)
    vb = torch.from_numpy(vf).to(cuda).to(torch.bfloat16)
    e8, _ = m.apply(var, v8)
    ef, _ = m.apply(var, vf)
    eb, _ = m.apply(var, vb)
    np.testing.assert_array_equal(e8, ef)
    np.testing.assert_array_equal(ef, eb.float().cpu().numpy() if torch.is_tensor(eb) else eb)
