"""MI355X parity of FactorizedVideoClassifier (encoders.py:583-653) through
the C-ABI (vp_classifier_*) against the NumPy oracle fp64.  Bars (written here; measured values
printed and recorded in DESIGN.md): fp32 logits / global embeddings max-abs 2e-5; bf16 logits
max-abs 3e-2 on O(1) logits with the L2-normalised global embedding within 1e-3."""

import numpy as np
import pytest
import torch

from oracle import videoprism_oracle as orc
from videoprism import encoders, models, params

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bf16", [False, True])
def test_classifier_reduced_depth(cuda, bf16):
    enc = dict(models.CONFIGS["videoprism_v1_base"])
    enc.update(num_spatial_layers=1, num_temporal_layers=1)
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoClassifier(encoder_params=enc,
                                                                                  num_classes=40),
                         fprop_dtype=torch.bfloat16 if bf16 else None)
    var = params.synthetic_params(enc, 4, specs=m.param_specs())
    video = np.random.default_rng(4).random((2, 2, 288, 288, 3), dtype=np.float32)
    logits, out = m.apply(var, video, return_intermediate=True)
    ref, rout = orc.video_classifier(var["params"], enc, video, return_intermediate=True)
    assert logits.shape == (2, 40)
    assert set(out) == {"spatial_features", "spatiotemporal_features", "global_embeddings"}
    el = np.abs(logits - ref).max()
    eg = np.abs(orc.l2_normalize(out["global_embeddings"]) - orc.l2_normalize(rout["global_embeddings"])).max()
    print(f"classifier {'bf16' if bf16 else 'f32'}: logits max-abs {el:.3e} (|logits| max "
          f"{np.abs(ref).max():.2f}), normalised global embedding {eg:.3e}")
    if bf16:
        assert el < 3e-2 and eg < 1e-3
    else:
        assert el < 2e-5 and np.abs(out["global_embeddings"] - rout["global_embeddings"]).max() < 2e-5


def test_classifier_large_u8(cuda):
    """Large dims (16 heads), uint8 frames, frame paddings; fp32."""
    enc = dict(models.CONFIGS["videoprism_v1_large"])
    enc.update(num_spatial_layers=1, num_temporal_layers=1)
    m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoClassifier(encoder_params=enc,
                                                                                  num_classes=7))
    var = params.synthetic_params(enc, 8, specs=m.param_specs())
    frames = np.random.default_rng(8).integers(0, 256, (1, 3, 288, 288, 3), dtype=np.uint8)
    fpad = np.array([[0.0, 0.0, 1.0]], np.float32)
    logits, _ = m.apply(var, frames, frame_paddings=fpad)
    ref, _ = orc.video_classifier(var["params"], enc, frames.astype(np.float32) / np.float32(255.0),
                                  frame_paddings=fpad)
    err = np.abs(logits - ref).max()
    print(f"classifier Large u8 f32: logits max-abs {err:.3e}")
    assert err < 2e-5
