"""GPU checks of the drop-in boundary's edges: attention without a logit cap or with a cap past
the max-free softmax's range (layers.py:586-589: cap <= 0 disables capping; FactorizedEncoder's
default cap is 0.0, encoders.py:407), the host engine's argument validation, the per-class kernel
symbol the bench's roofline keys its PMC record on, and the C-ABI RCCL all-gather (vp_allgather)
on a one-rank communicator, and empty batches (zero-size results, as the reference's JAX graph)."""

import os

import numpy as np
import pytest
import torch

from oracle import videoprism_oracle as orc
from videoprism import distributed, models, params

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    c = dict(models.CONFIGS["videoprism_v1_base"])
    c.update(num_spatial_layers=1, num_temporal_layers=1)
    c.update(kw)
    return c


def _model(cfg, bf16):
    return models.get_model(None, model_fn=lambda: models.encoders.FactorizedEncoder(**cfg),
                            fprop_dtype=torch.bfloat16 if bf16 else None)


def _pool_l2(e):
    m = e.astype(np.float64).mean(axis=1)
    return m / np.sqrt((m * m).sum(-1, keepdims=True) + 1e-12)


@pytest.mark.parametrize("cap", [0.0, 120.0])
def test_uncapped_and_large_cap_attention(cuda, cap):
    """bf16 with cap 0 (no tanh cap) or 120 (> 80: exp(cap) * S would overflow the max-free fp32
    softmax) runs the online-softmax kernel; fp32 likewise; both against the fp64 oracle."""
    cfg = _cfg(atten_logit_cap=cap)
    var = params.synthetic_params(cfg, seed=8)
    video = np.random.default_rng(8).random((1, 2, 288, 288, 3), dtype=np.float32)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, mode="f64")
    emb32, _ = _model(cfg, False).apply(var, video)
    e32 = np.abs(emb32 - ref).max()
    emb16, _ = _model(cfg, True).apply(var, video)
    assert np.isfinite(emb16).all()
    p16 = np.abs(_pool_l2(emb16) - _pool_l2(ref)).max()
    print(f"cap {cap}: f32 max-abs {e32:.3e}; bf16 pooled max-abs {p16:.3e}, token mean-abs "
          f"{np.abs(emb16 - ref).mean():.3e}")
    assert e32 <= 1e-5
    assert p16 <= 1e-3


def test_engine_rejects_bad_out_and_device(cuda):
    """Engine.forward hands raw pointers to the C-ABI: a wrong-shaped, strided, wrong-dtype or
    off-device `out` / `video` is refused before any launch."""
    cfg = _cfg()
    var = params.synthetic_params(cfg, seed=1)
    eng = _model(cfg, True).engine(var, 0)
    video = torch.rand((1, 2, 288, 288, 3), device=cuda).to(torch.bfloat16)
    good = torch.empty((1, 512, 768), device=cuda, dtype=torch.bfloat16)
    eng.forward(video, out=good)
    for bad in (torch.empty((1, 511, 768), device=cuda, dtype=torch.bfloat16),
                torch.empty((1, 768, 512), device=cuda, dtype=torch.bfloat16).transpose(1, 2),
                torch.empty((1, 512, 768), device=cuda, dtype=torch.float16),
                torch.empty((1, 512, 768), dtype=torch.bfloat16)):
        with pytest.raises(ValueError):
            eng.forward(video, out=bad)
    with pytest.raises(ValueError):
        eng.forward(video.cpu(), out=good)


def test_profile_kernel_symbol(cuda):
    """vp_profile_kernel_name names the kernel behind each profiled class (the key of the bench's
    PMC traffic record)."""
    cfg = _cfg()
    var = params.synthetic_params(cfg, seed=1)
    eng = _model(cfg, True).engine(var, 0)
    video = torch.rand((2, 2, 288, 288, 3), device=cuda).to(torch.bfloat16)
    eng.profile_enable(64)
    eng.forward(video)
    torch.cuda.synchronize()
    eng.profile_read()
    eng.profile_enable(0)
    names = {c: eng.kernel_name(c) for c in ("gemm_ffn1_gelu", "gemm_qkv", "attention_spatial")}
    print(names)
    assert names["gemm_ffn1_gelu"].startswith("gemm_bf16_w4_kernel<16")  # EPI_GELU_BF16_LN_BLK
    assert names["gemm_qkv"].startswith("gemm_bf16_w4_kernel<8")
    assert names["attention_spatial"].startswith("attn_spatial_kernel<")


def test_rccl_allgather_one_rank(cuda):
    """The C-ABI collective on real hardware: a one-rank RCCL communicator bootstrapped through
    torch.distributed (gloo store), vp_allgather of fp32 and bf16 rows."""
    import socket
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        comm = distributed.Communicator(0)
        for dt in (torch.float32, torch.bfloat16):
            x = torch.randn(4, 768, device=cuda).to(dt)
            y = comm.all_gather_rows(x)
            torch.cuda.synchronize()
            assert y.shape == (4, 768) and torch.equal(x, y)
        comm.close()
    finally:
        dist.destroy_process_group()


def test_allgather_side_stream_ordering(cuda):
    """Communicator.all_gather_rows on an explicit side stream: the rows are produced on the current
    stream by a long chain of kernels right before the call, and the result is consumed on the
    current stream right after it, with no synchronisation by the caller.  The gather must see the
    finished rows (the side stream waits for the current one) and the consumer the finished gather
    (the current stream waits for the side one); repeated with fresh allocations so a reuse of
    recorded memory would show.  (Uneven shards need world > 1: tests/test_distributed_cpu.py.)"""
    import socket

    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with distributed.Communicator(0) as comm:
            side = torch.cuda.Stream(device=cuda)
            big = torch.randn(4096, 4096, device=cuda)
            for it in range(4):
                x = torch.zeros(64, 768, device=cuda)
                for _ in range(8):  # keeps the current stream busy for a while
                    big = (big @ big).clamp_(-1.0, 1.0)
                x += float(it + 1)
                x += big[:64, :768] * 0.0
                y = comm.all_gather_rows(x, stream=side, counts=[64])
                z = y * 2.0  # consumed on the current stream
                del x
                torch.cuda.synchronize()
                assert torch.equal(z, torch.full_like(z, 2.0 * (it + 1))), it
    finally:
        dist.destroy_process_group()


def test_bench_base_step_world1_gather_vs_fixture(cuda):
    """bench.py's real base step at world 1 -- Engine.forward -> op_pool_l2 -> the library's RCCL
    gather (Communicator.all_gather_rows over a one-rank communicator, bootstrapped through a gloo
    group as bench.py does) -- on the g6 fixture clip (full Base, T = 16) among 3 others: the
    gathered row of the fixture clip is within 1e-3 of the fixture's fp64 pooled vector."""
    import socket

    import torch.distributed as dist

    from videoprism import _native
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "g6_base_t16.npz"),
                allow_pickle=False)
    cfg = models.CONFIGS["videoprism_v1_base"]
    var = params.synthetic_params(cfg, seed=int(g["param_seed"]))
    eng = models.get_model("videoprism_public_v1_base", fprop_dtype=torch.bfloat16).engine(var, 0)
    video0 = np.random.default_rng(int(g["video_seed"])).random((1, 16, 288, 288, 3), dtype=np.float32)
    gen = torch.Generator(device=cuda).manual_seed(1000)
    video = torch.rand((4, 16, 288, 288, 3), generator=gen, device=cuda).to(torch.bfloat16)
    video[2] = torch.from_numpy(video0[0]).to(cuda).to(torch.bfloat16)
    out = torch.empty((4, 4096, 768), dtype=torch.bfloat16, device=cuda)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with distributed.Communicator(0) as comm:
            eng.forward(video, out=out)
            rows = comm.all_gather_rows(_native.op_pool_l2(out), counts=[4])
            torch.cuda.synchronize()
        assert rows.shape == (4, 768) and rows.dtype == torch.float32
        err = np.abs(rows[2].double().cpu().numpy() - g["pooled_f64"][0]).max()
        print(f"bench base step, world 1: gathered pooled row of the fixture clip max-abs {err:.3e}")
        assert err <= 1e-3
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bf16", [False, True])
def test_empty_batch_zero_size_results(cuda, bf16):
    """B = 0 clips (and Q = 0 text queries): the reference's JAX graph maps zero-size arrays to
    zero-size results (encoders.py:436 reshapes [0, T, H, W, 3] to [0, H, W, 3]; every later op is
    shape-polymorphic), so the drop-in returns [0, T*N, D] embeddings (and zero-size intermediates,
    logits, video / text embeddings) instead of an error; the geometry and frame_paddings checks still
    apply, and a following non-empty forward is unaffected."""
    dt = torch.bfloat16 if bf16 else None
    cfg = _cfg()
    var = params.synthetic_params(cfg, seed=3)
    mdl = _model(cfg, bf16)
    emb, out = mdl.apply(var, np.zeros((0, 2, 288, 288, 3), np.float32), return_intermediate=True,
                         frame_paddings=np.zeros((0, 2), np.float32))
    assert emb.shape == (0, 512, 768) and out["spatial_features"].shape == (0, 512, 768)
    with pytest.raises(ValueError):
        mdl.apply(var, np.zeros((0, 2, 280, 280, 3), np.float32))  # 280 % 18 != 0, as the reference
    with pytest.raises(AssertionError):
        mdl.apply(var, np.zeros((0, 2, 288, 288, 3), np.float32), frame_paddings=np.zeros((1, 2), np.float32))
    video = np.random.default_rng(3).random((1, 2, 288, 288, 3), dtype=np.float32)
    e1, _ = mdl.apply(var, video)
    ref, _ = orc.factorized_encoder(var["params"], video, cfg, mode="f64")
    assert np.abs(_pool_l2(e1) - _pool_l2(ref)).max() <= (1e-3 if bf16 else 1e-5)

    ccfg = dict(models.CONFIGS["videoprism_lvt_v1_base"])
    ccfg.update(num_spatial_layers=1, num_temporal_layers=1, num_auxiliary_layers=1, num_unimodal_layers=1,
                vocabulary_size=100)
    clip = models.get_model(None, model_fn=lambda: models.encoders.FactorizedVideoCLIP(**ccfg), fprop_dtype=dt)
    cvar = params.synthetic_params(ccfg, seed=3, specs=params.clip_leaf_specs(ccfg))
    v, t, cout = clip.apply(cvar, np.zeros((0, 2, 288, 288, 3), np.float32), np.zeros((0, 16), np.int32),
                            np.zeros((0, 16), np.float32), return_intermediate=True)
    assert v.shape == (0, 768) and t.shape == (0, 768)
    assert cout["frame_embeddings"].shape == (0, 2, 768) and cout["spatiotemporal_features"].shape == (0, 512, 768)

    enc = dict(models.CONFIGS["videoprism_v1_base"])
    enc.update(num_spatial_layers=1, num_temporal_layers=1)
    cls = models.get_model(None, model_fn=lambda: models.encoders.FactorizedVideoClassifier(encoder_params=enc,
                                                                                          num_classes=5),
                           fprop_dtype=dt)
    kvar = params.synthetic_params(enc, 3, specs=cls.param_specs())
    logits, kout = cls.apply(kvar, np.zeros((0, 2, 288, 288, 3), np.uint8), return_intermediate=True)
    assert logits.shape == (0, 5) and kout["global_embeddings"].shape == (0, 768)
