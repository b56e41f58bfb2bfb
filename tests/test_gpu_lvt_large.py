"""configs[4]'s per-rank workload at full depth: the LvT-Large video-text model
(`videoprism_lvt_v1_large`: 24 + 4 vision layers, 2 auxiliary layers whose attention spans all
4096 tokens of a 16-frame clip at D = 1024, the contrastive pooler, 12 causal text layers;
encoders.py:762-910, models.py:131-145) in bf16 on one MI355X.

  * B = 1 against the fp64 oracle fixture tests/golden/g8_lvt_large_t16.npz (make_golden.py
    g8, same seeds): video embedding, both text embeddings and the similarity video_emb @
    text_emb.T (README.md:81) within the reference's own 1e-3 bar (verify_clip_models.py:237);
  * the bench's per-rank batch B = 32 (bench.py --workload lvt_large): clips 0 and 31 bitwise
    equal to their B = 1 runs, clip 0 being the fixture clip, whose similarity row stays within
    1e-3 of the fixture.

The fixture also holds the oracle's emulation of the reference's own bf16 graph; its distance
from fp64 is printed beside ours.  Parity unpinned by the reference (JAX absent).
"""

import os

import numpy as np
import pytest
import torch

from videoprism import _native as nat
from videoprism import models, params

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "g8_lvt_large_t16.npz")


@pytest.fixture(scope="module")
def lvt_large(cuda):
    g = np.load(GOLD, allow_pickle=False)
    cfg = dict(models.CONFIGS[str(g["cfg"])])
    cfg["vocabulary_size"] = int(g["vocabulary_size"])
    var = params.synthetic_params(cfg, seed=int(g["param_seed"]), specs=params.clip_leaf_specs(cfg))
    mdl = models.get_model("videoprism_lvt_public_v1_large", fprop_dtype=torch.bfloat16)
    assert mdl.vocabulary_size == cfg["vocabulary_size"]
    eng = mdl.engine(var, torch.cuda.current_device())
    video = np.random.default_rng(int(g["video_seed"])).random((1, 16, 288, 288, 3), dtype=np.float32)
    ids = torch.from_numpy(g["text_token_ids"]).to(cuda)
    pads = torch.from_numpy(g["text_paddings"]).to(cuda)
    temb = eng.encode_text(ids, pads)
    torch.cuda.synchronize()
    return g, eng, torch.from_numpy(video).to(cuda).to(torch.bfloat16), temb


def _report(tag, got, g, name):
    err = np.abs(got - g[f"{name}_f64"]).max()
    emu = np.abs(g[f"{name}_bf16"] - g[f"{name}_f64"]).max()
    print(f"{tag} {name}: max-abs vs fp64 {err:.3e} (reference bf16 emulation {emu:.3e})")
    return err


def test_lvt_large_full_depth_vs_oracle(lvt_large):
    g, eng, video, temb = lvt_large
    vemb, femb, _, _ = eng.encode_video(video, want_frames=True)
    sim = nat.op_similarity(vemb, temb)
    torch.cuda.synchronize()
    ev = _report("LvT-L B=1", vemb.cpu().numpy(), g, "video_emb")
    et = _report("LvT-L B=1", temb.cpu().numpy(), g, "text_emb")
    es = _report("LvT-L B=1", sim.cpu().numpy(), g, "similarity")
    ef = _report("LvT-L B=1", femb.cpu().numpy(), g, "frame_emb")
    np.testing.assert_allclose(np.linalg.norm(vemb.cpu().numpy(), axis=-1), 1.0, rtol=1e-5)
    assert ev <= 1e-3 and et <= 1e-3 and es <= 1e-3, (ev, et, es)
    assert ef <= 2e-3, ef


def test_lvt_large_bench_batch_bitwise(lvt_large, cuda):
    g, eng, video0, temb = lvt_large
    B = 32
    gen = torch.Generator(device=cuda).manual_seed(123)
    batch = torch.rand((B, 16, 288, 288, 3), generator=gen, device=cuda).to(torch.bfloat16)
    batch[0] = video0[0]
    full = eng.encode_video(batch)[0].clone()
    sim = nat.op_similarity(full, temb)
    torch.cuda.synchronize()
    for b in (0, B - 1):
        one = eng.encode_video(batch[b:b + 1].contiguous())[0]
        torch.cuda.synchronize()
        assert torch.equal(one[0], full[b]), b
    es = _report("LvT-L B=32 clip 0", sim[:1].cpu().numpy(), g, "similarity")
    assert sim.shape == (B, 2)
    assert es <= 1e-3, es
