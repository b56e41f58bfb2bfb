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
