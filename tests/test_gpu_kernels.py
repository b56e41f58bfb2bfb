"""Op-level parity of the HIP kernels (through the C-ABI op entry points) against
plain PyTorch fp32/fp64 references and the NumPy oracle.

Tolerances:
  * bf16 GEMM: operands are exactly representable bf16, accumulation fp32 -> fp32 outputs
    agree with an fp64 matmul of the same operands to ~1e-6 relative (1e-4 abs at O(1)
    scale); bf16 outputs additionally carry one bf16 rounding (rtol 2^-8).
  * fp32 GEMM (v_mfma_f32_16x16x4_f32): 2e-5 abs at O(1) scale for K <= 3072.
  * bf16 attention: P is rounded to bf16 before P.V (as the reference's bf16 mode rounds
    probs, layers.py:654): 1e-2 abs on O(1) values.
"""

import numpy as np
import pytest
import torch

from videoprism import _native as nat
from oracle import videoprism_oracle as orc

pytestmark = pytest.mark.gpu


def _bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 768), (1024, 2304, 768), (256, 768, 3072), (512, 1024, 1024)])
def test_gemm_bf16_store(cuda, M, N, K):
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda) * 0.1
    ab, wb = _bf(a), _bf(w)
    ref = ab.double() @ wb.double().T + b.double()
    out = nat.op_gemm(ab, wb, b, nat.EPI_STORE)
    torch.cuda.synchronize()
    assert out.dtype == torch.bfloat16
    err = (out.double() - ref).abs()
    assert torch.all(err <= 2 ** -8 * ref.abs() + 1e-3), float(err.max())


@pytest.mark.parametrize("M,N,K", [(512, 3072, 768), (256, 256, 128)])
def test_gemm_bf16_gelu_rowpad(cuda, M, N, K):
    g = torch.Generator(device="cpu").manual_seed(7)
    a = _bf(torch.randn(M, K, generator=g)).to(cuda)
    w = _bf(torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    pad = (torch.rand(M, generator=g) < 0.25).float().to(cuda)
    out = nat.op_gemm(a, w, b, nat.EPI_GELU, rowpad=pad)
    torch.cuda.synchronize()
    y = a.double() @ w.double().T + b.double()
    ref = 0.5 * y * (1 + torch.erf(y / 2 ** 0.5)) * (1 - pad.double())[:, None]
    err = (out.double() - ref).abs()
    assert torch.all(err <= 2 ** -8 * ref.abs() + 1e-3), float(err.max())


@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (256, 768, 3072)])
def test_gemm_bf16_resid_inplace(cuda, M, N, K):
    g = torch.Generator(device="cpu").manual_seed(11)
    a = _bf(torch.randn(M, K, generator=g)).to(cuda)
    w = _bf(torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    x = torch.randn(M, N, generator=g).to(cuda)
    pad = (torch.rand(M, generator=g) < 0.25).float().to(cuda)
    ref = x.double() + (a.double() @ w.double().T + b.double()) * (1 - pad.double())[:, None]
    nat.op_gemm(a, w, b, nat.EPI_RESID, out=x, resid=x, rowpad=pad)
    torch.cuda.synchronize()
    assert float((x.double() - ref).abs().max()) < 1e-4


def test_gemm_bf16_pos(cuda):
    M, N, K = 1024, 768, 1024
    g = torch.Generator(device="cpu").manual_seed(5)
    a = _bf(torch.rand(M, K, generator=g)).to(cuda)
    w = _bf(torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    pos = torch.randn(256, N, generator=g).to(cuda)
    out = nat.op_gemm(a, w, b, nat.EPI_POS, pos=pos)
    torch.cuda.synchronize()
    ref = a.double() @ w.double().T + b.double() + pos.double().repeat(M // 256, 1)
    assert float((out.double() - ref).abs().max()) < 1e-4


@pytest.mark.parametrize("epi", [nat.EPI_RESID_BF16, nat.EPI_RESID_FFN_BF16])
def test_gemm_bf16_resid_bf16_stream(cuda, epi):
    """bf16 residual stream (fprop_dtype bf16 keeps x in bf16, models.py:301-302): out =
    bf16(x + (a.w^T + b) * keep), one rounding -> |err| <= 2^-8 |ref| + fp32-accumulation slack."""
    M, N, K = 2048, 768, 3072 if epi == nat.EPI_RESID_FFN_BF16 else 768
    g = torch.Generator(device="cpu").manual_seed(21 + epi)
    a = _bf(torch.randn(M, K, generator=g)).to(cuda)
    w = _bf(torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    x = _bf(torch.randn(M, N, generator=g) * 4).to(cuda)
    pad = (torch.rand(M, generator=g) < 0.25).float().to(cuda)
    ref = x.double() + (a.double() @ w.double().T + b.double()) * (1 - pad.double())[:, None]
    nat.op_gemm(a, w, b, epi, out=x, resid=x, rowpad=pad)
    torch.cuda.synchronize()
    assert x.dtype == torch.bfloat16
    err = (x.double() - ref).abs()
    assert bool((err <= 2 ** -8 * ref.abs() + 1e-4).all()), float(err.max())


def test_gemm_bf16_pos_bf16(cuda):
    M, N, K = 1024, 768, 1024
    g = torch.Generator(device="cpu").manual_seed(6)
    a = _bf(torch.rand(M, K, generator=g)).to(cuda)
    w = _bf(torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    pos = torch.randn(256, N, generator=g).to(cuda)
    out = nat.op_gemm(a, w, b, nat.EPI_POS_BF16, pos=pos)
    torch.cuda.synchronize()
    assert out.dtype == torch.bfloat16
    ref = a.double() @ w.double().T + b.double() + pos.double().repeat(M // 256, 1)
    err = (out.double() - ref).abs()
    assert bool((err <= 2 ** -8 * ref.abs() + 1e-4).all()), float(err.max())


# both bf16 GEMM kernels on persistent shapes: tiles > CUs (several tiles per workgroup, so the
# K-tile stream crosses tile boundaries), tile counts not divisible by 8 XCDs, K = 1..48 K-tiles;
# (4096, 3072, 768) has W = 4.7 MB > an XCD's L2, so the 4-wave kernel runs it in the N-tile
# grouped tile order (w4_ngrp: groups of 6 N-tiles, 192 workgroups) -- the same order as ffn_layer1;
# (1280, 768, 704): odd counts everywhere -- 5 M-blocks, 3 N-tiles, 11 K-tiles (the K-tile stream's
# two-buffer / S3 three-buffer rotation ends on an odd phase)
KERNEL_SHAPES = [(16384, 2304, 768), (32768, 768, 3072), (2304, 1536, 64), (512, 256, 1024),
                 (4096, 3072, 768), (1280, 768, 704)]


@pytest.mark.parametrize("M,N,K", KERNEL_SHAPES)
@pytest.mark.parametrize("epi", [nat.EPI_STORE, nat.EPI_GELU, nat.EPI_RESID, nat.EPI_POS,
                                 nat.EPI_RESID_FFN, nat.EPI_RESID_BF16, nat.EPI_POS_BF16,
                                 nat.EPI_RESID_FFN_BF16])
def test_gemm_kernels_bitwise_equal(cuda, M, N, K, epi):
    """The 4-wave and 8-wave kernels sum each output's K products in the same order (k-halves of
    32 in sequence, fp32 MFMA accumulation), so they must agree bit for bit on every epilogue;
    one of them is additionally checked against fp64."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    a = _bf(torch.randn(M, K, generator=g)).to(cuda)
    w = _bf(torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    pad = (torch.rand(M, generator=g) < 0.2).float().to(cuda)
    pos = torch.randn(256, N, generator=g).to(cuda) if epi in (nat.EPI_POS, nat.EPI_POS_BF16) else None
    f32_out = epi in (nat.EPI_RESID, nat.EPI_POS, nat.EPI_RESID_FFN)
    resid = epi in (nat.EPI_RESID, nat.EPI_RESID_FFN, nat.EPI_RESID_BF16, nat.EPI_RESID_FFN_BF16)
    x0 = torch.randn(M, N, generator=g).to(cuda)
    outs = {}
    for which in (4, 8):
        if resid:
            o = x0.clone() if f32_out else x0.to(torch.bfloat16)
        else:
            o = torch.empty(M, N, device=cuda, dtype=torch.float32 if f32_out else torch.bfloat16)
        nat.dev_gemm_kernel(which, a, w, b, epi, o, resid=o if resid else None, pos=pos,
                            rowpad=pad if epi != nat.EPI_POS and epi != nat.EPI_POS_BF16 else None)
        outs[which] = o
    torch.cuda.synchronize()
    assert torch.equal(outs[4], outs[8])
    y = a.double() @ w.double().T + b.double()
    keep = (1 - pad.double())[:, None]
    if epi == nat.EPI_STORE:
        ref = y
    elif epi == nat.EPI_GELU:
        ref = 0.5 * y * (1 + torch.erf(y / 2 ** 0.5)) * keep
    elif epi in (nat.EPI_POS, nat.EPI_POS_BF16):
        ref = y + pos.double().repeat(M // 256, 1)
    else:
        xr = x0.double() if f32_out else x0.to(torch.bfloat16).double()
        ref = xr + y * keep
    err = (next(iter(outs.values())).double() - ref).abs()
    tol = (1e-4 if f32_out else 2 ** -8 * ref.abs() + 1e-4) + 5e-6 * K ** 0.5
    assert bool((err <= tol).all()), float(err.max())


@pytest.mark.parametrize("M,N,K", [(64, 64, 256), (768, 1024, 1024), (768, 4096, 1024), (768, 1024, 4096),
                                   (576, 768, 3072)])
@pytest.mark.parametrize("epi", [nat.EPI_STORE, nat.EPI_GELU, 13, nat.EPI_RESID, nat.EPI_RESID_FFN,
                                 nat.EPI_RESID_BF16, nat.EPI_RESID_FFN_BF16])
def test_gemm_small_m_kernel(cuda, M, N, K, epi):
    """gemm_bf16_small.hip (the text tower's GEMMs: 64 x 64 tiles, K split over 4 waves, partials summed
    in LDS in wave order) against fp64 on every epilogue it takes (13 = ReLU, encoders.py:743), with
    padded rows; the shapes are the LvT-Large / Base text tower's at 8 queries (M = 768; 576 = 9 x 64)."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    a = _bf(torch.randn(M, K, generator=g)).to(cuda)
    w = _bf(torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    pad = (torch.rand(M, generator=g) < 0.2).float().to(cuda)
    f32_out = epi in (nat.EPI_RESID, nat.EPI_RESID_FFN)
    resid = epi in (nat.EPI_RESID, nat.EPI_RESID_FFN, nat.EPI_RESID_BF16, nat.EPI_RESID_FFN_BF16)
    x0 = torch.randn(M, N, generator=g).to(cuda)
    if resid:
        o = x0.clone() if f32_out else x0.to(torch.bfloat16)
    else:
        o = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    rp = None if epi == nat.EPI_STORE else pad
    nat.dev_gemm_kernel(1, a, w, b, epi, o, resid=o if resid else None, rowpad=rp)
    torch.cuda.synchronize()
    y = a.double() @ w.double().T + b.double()
    keep = (1 - pad.double())[:, None]
    if epi == nat.EPI_STORE:
        ref = y
    elif epi == nat.EPI_GELU:
        ref = 0.5 * y * (1 + torch.erf(y / 2 ** 0.5)) * keep
    elif epi == 13:
        ref = y.clamp(min=0) * keep
    else:
        xr = x0.double() if f32_out else x0.to(torch.bfloat16).double()
        ref = xr + y * keep
    err = (o.double() - ref).abs()
    tol = (1e-4 if f32_out else 2 ** -8 * ref.abs() + 1e-4) + 5e-6 * K ** 0.5
    assert bool((err <= tol).all()), float(err.max())


def test_gemm_small_m_rejects_unsupported(cuda):
    a = torch.zeros(64, 192, dtype=torch.bfloat16, device=cuda)  # K % 256 != 0
    w = torch.zeros(64, 192, dtype=torch.bfloat16, device=cuda)
    b = torch.zeros(64, device=cuda)
    o = torch.empty(64, 64, dtype=torch.bfloat16, device=cuda)
    with pytest.raises(Exception, match="small-M GEMM"):
        nat.dev_gemm_kernel(1, a, w, b, nat.EPI_STORE, o)


def test_gemm_bf16_asymmetric_identity(cuda):
    """A = I with an asymmetric W catches a transposed C write (guide §3)."""
    M = N = K = 256
    a = _bf(torch.eye(M)).to(cuda)
    w = _bf(torch.arange(N * K, dtype=torch.float32).reshape(N, K) % 97 - 48).to(cuda)
    b = torch.zeros(N, device=cuda)
    out = nat.op_gemm(a, w, b, nat.EPI_RESID, out=torch.zeros(M, N, device=cuda),
                      resid=torch.zeros(M, N, device=cuda))
    torch.cuda.synchronize()
    assert torch.equal(out, w.float().T.contiguous())


@pytest.mark.parametrize("epi", [nat.EPI_STORE, nat.EPI_GELU, nat.EPI_RESID, nat.EPI_POS])
def test_gemm_f32(cuda, epi):
    M, N, K = 512, 768, 3072 if epi == nat.EPI_RESID else 768
    g = torch.Generator(device="cpu").manual_seed(epi)
    a = torch.randn(M, K, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    pad = (torch.rand(M, generator=g) < 0.25).float().to(cuda)
    x = torch.randn(M, N, generator=g).to(cuda)
    pos = torch.randn(256, N, generator=g).to(cuda)
    y = a.double() @ w.double().T + b.double()
    if epi == nat.EPI_STORE:
        out, ref = nat.op_gemm(a, w, b, epi), y
    elif epi == nat.EPI_GELU:
        out = nat.op_gemm(a, w, b, epi, rowpad=pad)
        ref = 0.5 * y * (1 + torch.erf(y / 2 ** 0.5)) * (1 - pad.double())[:, None]
    elif epi == nat.EPI_RESID:
        ref = x.double() + y * (1 - pad.double())[:, None]
        out = nat.op_gemm(a, w, b, epi, out=x, resid=x, rowpad=pad)
    else:
        out = nat.op_gemm(a, w, b, epi, pos=pos)
        ref = y + pos.double().repeat(M // 256, 1)
    torch.cuda.synchronize()
    assert float((out.double() - ref).abs().max()) < 2e-5


def _qkv(num_seq, S, heads, seed, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    D = heads * 64
    q = torch.randn(num_seq * S, D, generator=g) * scale * 0.125 * 8
    k = torch.randn(num_seq * S, D, generator=g) * scale
    v = torch.randn(num_seq * S, D, generator=g)
    return torch.cat([q, k, v], dim=1)


def _oracle_attention(qkv, num_seq, S, heads, cap, key_pad=None):
    D = heads * 64
    x = qkv.double().cpu().numpy().reshape(num_seq, S, 3, heads, 64)
    q = x[:, :, 0].transpose(0, 2, 1, 3).reshape(num_seq * heads, S, 64)
    k = x[:, :, 1].transpose(0, 2, 1, 3).reshape(num_seq * heads, S, 64)
    v = x[:, :, 2].transpose(0, 2, 1, 3).reshape(num_seq * heads, S, 64)
    kp = None
    if key_pad is not None:
        kp = np.repeat(key_pad.cpu().numpy().reshape(num_seq, 1, S), heads, axis=1).reshape(-1, S)
    o = orc.capped_softmax_attention(q, k, v, cap, kp)
    return o.reshape(num_seq, heads, S, 64).transpose(0, 2, 1, 3).reshape(num_seq * S, D)


# scale 0.125 keeps the logits in the one-transcendental polynomial range (vp_common.h
# capped_exp16); the larger scales exercise the exact path
@pytest.mark.parametrize("S,num_seq,heads,scale", [(256, 3, 12, 1.0), (256, 2, 16, 4.0), (256, 2, 12, 0.125),
                                                   (16, 40, 12, 1.0), (8, 9, 12, 3.0), (5, 7, 16, 1.0),
                                                   (17, 9, 12, 1.0), (32, 10, 12, 3.0), (40, 5, 16, 1.0),
                                                   (64, 9, 12, 1.0), (100, 3, 12, 4.0), (128, 5, 16, 1.0),
                                                   (200, 3, 12, 1.0)])
def test_attention_bf16(cuda, S, num_seq, heads, scale):
    qkv = _bf(_qkv(num_seq, S, heads, S + num_seq, scale)).to(cuda)
    out = nat.op_attention(qkv, num_seq, S, heads, 50.0)
    torch.cuda.synchronize()
    ref = _oracle_attention(qkv, num_seq, S, heads, 50.0)
    err = np.abs(out.double().cpu().numpy() - ref)
    # bound: bf16 rounding of the output (2^-9 |o|) + of each numerator before P.V
    # (2^-9 * max|v|), doubled for accumulation slack
    vmax = float(qkv[:, 2 * heads * 64:].float().abs().max())
    assert np.all(err <= 2 ** -8 * (np.abs(ref) + vmax)), err.max()
    assert err.mean() < 2e-3, err.mean()


@pytest.mark.parametrize("S,num_seq,heads,cap", [(256, 2, 12, 80.0), (4096, 1, 2, 80.0),
                                                 (256, 2, 12, 50.0), (4096, 1, 2, 50.0)])
def test_attention_bf16_saturated_logits_large_v(cuda, S, num_seq, heads, cap):
    """Saturated logits (|q.k| >> cap, so cap*tanh(.) sits at +-cap) with |v| ~ 200: the max-free
    kernels' unnormalised fp32 O = sum exp(l) v would overflow for cap = 80 (e^80 * S * |v| >
    FLT_MAX), so caps above 50 must take the online-softmax kernel; at cap = 50 the fast kernels
    stay finite.  Both against the fp64 oracle."""
    qkv = _qkv(num_seq, S, heads, 4242 + S, 40.0)
    qkv[:, 2 * heads * 64:] *= 200.0
    qkv = _bf(qkv).to(cuda)
    out = nat.op_attention(qkv, num_seq, S, heads, cap)
    torch.cuda.synchronize()
    o = out.double().cpu().numpy()
    assert np.isfinite(o).all()
    ref = _oracle_attention(qkv, num_seq, S, heads, cap)
    vmax = float(qkv[:, 2 * heads * 64:].float().abs().max())
    err = np.abs(o - ref)
    print(f"cap {cap} S {S}: max-abs {err.max():.3e} (max|v| {vmax:.0f})")
    assert np.all(err <= 2 ** -8 * (np.abs(ref) + vmax)), err.max()


@pytest.mark.parametrize("S,num_seq", [(256, 3), (16, 10), (8, 6), (40, 11), (64, 9), (130, 3)])
def test_attention_bf16_key_padding(cuda, S, num_seq):
    heads = 12
    qkv = _bf(_qkv(num_seq, S, heads, 3)).to(cuda)
    g = torch.Generator(device="cpu").manual_seed(9)
    if S == 256:  # spatial stage: a padded frame pads all of its keys
        kp = torch.zeros(num_seq, S)
        kp[1] = 1.0
    else:
        kp = (torch.rand(num_seq, S, generator=g) < 0.4).float()
        kp[0] = 1.0  # fully padded sequence -> uniform attention
    kp = kp.reshape(-1).to(cuda)
    out = nat.op_attention(qkv, num_seq, S, heads, 50.0, key_pad=kp)
    torch.cuda.synchronize()
    ref = _oracle_attention(qkv, num_seq, S, heads, 50.0, kp.reshape(num_seq, S))
    err = np.abs(out.double().cpu().numpy() - ref)
    vmax = float(qkv[:, 2 * heads * 64:].float().abs().max())
    assert np.all(err <= 2 ** -8 * (np.abs(ref) + vmax)), err.max()


@pytest.mark.parametrize("S,num_seq,heads", [(256, 2, 12), (16, 20, 12), (4, 3, 16)])
def test_attention_f32(cuda, S, num_seq, heads):
    qkv = _qkv(num_seq, S, heads, 17, 2.0).to(cuda)
    kp = torch.zeros(num_seq, S)
    kp[-1, : S // 2] = 1.0
    out = nat.op_attention(qkv, num_seq, S, heads, 50.0, key_pad=kp.reshape(-1).to(cuda))
    torch.cuda.synchronize()
    ref = _oracle_attention(qkv, num_seq, S, heads, 50.0, kp)
    # logits here reach |q.k| ~ 100 (scale 2): fp32 ulp there is ~8e-6, so the probabilities
    # carry ~1e-5 relative error by construction; bound 3e-5 on O(1) outputs.
    assert np.abs(out.double().cpu().numpy() - ref).max() < 3e-5


@pytest.mark.parametrize("S,num_seq,heads,scale,pad,cap", [
    (256, 5, 12, 1.0, None, 50.0), (256, 5, 16, 0.125, None, 50.0), (256, 5, 12, 4.0, "frame", 50.0),
    (256, 5, 16, 1.0, "random", 50.0), (256, 3, 12, 2.0, "random", 80.0), (256, 3, 12, 1.0, None, 0.0),
    (128, 4, 12, 1.0, "random", 50.0), (200, 3, 16, 1.0, None, 50.0), (300, 2, 12, 1.0, "random", 50.0),
    (520, 2, 12, 2.0, None, 50.0), (1000, 1, 16, 0.5, "random", 50.0), (2048, 1, 12, 1.0, None, 50.0),
    (300, 2, 12, 1.0, None, 0.0)])
def test_attention_f32_mfma(cuda, S, num_seq, heads, scale, pad, cap):
    """fp32 attention (fprop_dtype=float32): S >= 128 with 0 < cap <= 50 takes the MFMA kernel
    (attn_f32_mfma_kernel: 256-query blocks, 128-key chunks, a partial last block / chunk when S % 256 != 0),
    cap 80 / no cap the generic online-softmax kernels; key paddings as the reference's
    where(mask, logits, -0.7 FLT_MAX): a padded frame (every key: uniform weights) or random keys with one
    fully padded sequence.  Against the fp64 oracle; bar 3e-5 relative to max(1, |o|), test_attention_f32's:
    logits reach |q.k| ~ 100 at scale 2 - 4, where the fp32 rounding of the logit alone moves a probability
    ~1e-5 relative."""
    qkv = _qkv(num_seq, S, heads, 31 + heads + S, scale).to(cuda)
    kp = None
    if pad == "frame":
        kp = torch.zeros(num_seq, S)
        kp[2] = 1.0
    elif pad == "random":
        g = torch.Generator(device="cpu").manual_seed(5)
        kp = (torch.rand(num_seq, S, generator=g) < 0.3).float()
        kp[-1] = 1.0
    out = nat.op_attention(qkv, num_seq, S, heads, cap, key_pad=None if kp is None else kp.reshape(-1).to(cuda))
    torch.cuda.synchronize()
    ref = _oracle_attention(qkv, num_seq, S, heads, cap, kp)
    err = np.abs(out.double().cpu().numpy() - ref)
    print(f"f32 S={S} heads {heads} scale {scale} pad {pad} cap {cap}: max-abs {err.max():.3e}")
    assert np.all(err <= 3e-5 * np.maximum(1.0, np.abs(ref))), err.max()


@pytest.mark.parametrize("D,perm", [(768, nat.PERM_NONE), (768, nat.PERM_BTN_TO_BNT),
                                    (1024, nat.PERM_BNT_TO_BTN)])
@pytest.mark.parametrize("out_bf16", [False, True])
@pytest.mark.parametrize("in_bf16", [False, True])
def test_layernorm(cuda, D, perm, out_bf16, in_bf16):
    B, T, N = 2, 4, 256
    g = torch.Generator(device="cpu").manual_seed(D + perm)
    x = (torch.randn(B * T * N, D, generator=g) * 3 + 1).to(cuda)
    if in_bf16:  # bf16 residual stream: the reference value is the LN of the bf16 input
        x = x.to(torch.bfloat16)
    scale = torch.randn(D, generator=g) * 0.1
    bias = torch.randn(D, generator=g) * 0.1
    add = torch.randn(T, D, generator=g).to(cuda) if perm == nat.PERM_BTN_TO_BNT else None
    out = nat.op_layernorm(x, (1 + scale).to(cuda), bias.to(cuda),
                           torch.bfloat16 if out_bf16 else torch.float32, perm, T, N, add)
    torch.cuda.synchronize()
    xd = x.double().cpu().numpy()
    ref = orc.layer_norm(xd, scale.double().numpy(), bias.double().numpy(), orc.Numerics("f64"))
    if perm == nat.PERM_BTN_TO_BNT:
        ref = ref.reshape(B, T, N, D).transpose(0, 2, 1, 3) + add.double().cpu().numpy()[None, None]
        ref = ref.reshape(-1, D)
    elif perm == nat.PERM_BNT_TO_BTN:
        ref = ref.reshape(B, N, T, D).transpose(0, 2, 1, 3).reshape(-1, D)
    err = np.abs(out.double().cpu().numpy() - ref)
    tol = 2 ** -8 * np.abs(ref) + 1e-5 if out_bf16 else 2e-5
    assert np.all(err <= tol), err.max()


@pytest.mark.parametrize("in_bf16", [False, True])
def test_patchify(cuda, in_bf16):
    BT, H, P = 3, 288, 18
    g = torch.Generator(device="cpu").manual_seed(1)
    v = torch.rand(BT, H, H, 3, generator=g)
    if in_bf16:
        v = _bf(v)
    vd = v.to(cuda)
    out = nat.op_patchify(vd, P, 1024, torch.bfloat16)
    torch.cuda.synchronize()
    ref = orc.image_to_patch(v.float().numpy(), P).reshape(-1, P * P * 3)
    got = out.float().cpu().numpy()
    np.testing.assert_array_equal(got[:, P * P * 3:], 0)
    np.testing.assert_array_equal(got[:, : P * P * 3], orc.round_bf16(ref))


def test_pool_l2(cuda):
    g = torch.Generator(device="cpu").manual_seed(2)
    e = torch.randn(3, 4096, 768, generator=g).to(cuda)
    out = nat.op_pool_l2(e)
    torch.cuda.synchronize()
    m = e.double().mean(1)
    ref = m / torch.sqrt((m * m).sum(-1, keepdim=True) + 1e-12)
    assert float((out.double() - ref).abs().max()) < 1e-6


# ---- GEMM-folded LayerNorm (bf16 forward): EPI_*_LN consumers and EPI_*_ST producers ----

def _ln_ref(x, gamma1p, beta):
    """layers.py:208-270 in fp64: (x - mean) * rsqrt(var + 1e-6) * (1 + scale) + bias."""
    m = x.mean(-1, keepdim=True)
    v = ((x - m) ** 2).mean(-1, keepdim=True)
    return (x - m) / torch.sqrt(v + 1e-6) * gamma1p + beta


@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("frames,D", [(6, 768), (3, 1024)])
def test_qkv_spatial_attention_row_blocked_bitwise(cuda, masked, frames, D):
    """The spatial layers' q|k|v projection into the row-blocked layout (EPI_BF16_LN_BLK, rows of Wqkv /
    b' / c permuted within 32-row groups) and the spatial attention reading it are bitwise the row-major
    pair: q|k|v re-laid equal, attention output equal (with and without padded keys)."""
    M, NH = frames * 256, D // 64
    g = torch.Generator(device="cpu").manual_seed(frames + D + masked)
    x = _bf(torch.randn(M, D, generator=g) * 2 + 0.5)
    w = _bf(torch.randn(3 * D, D, generator=g) / D ** 0.5)
    b = torch.randn(3 * D, generator=g) * 0.1
    c = w.double().sum(1).float()
    xd = x.to(cuda)
    rs = torch.empty(M, 2, device=cuda)
    nat.dev_ln_stats(xd, M, D, rs, from_partials=False)
    perm = torch.from_numpy(nat.ffn1_blk_rows(3 * D))
    q_rm = torch.empty(M, 3 * D, device=cuda, dtype=torch.bfloat16)
    q_bk = torch.empty_like(q_rm)
    nat.dev_gemm_ln(xd, w.to(cuda), b.to(cuda), nat.EPI_BF16_LN, q_rm, ln_rs=rs, ln_c=c.to(cuda))
    nat.dev_gemm_ln(xd, w[perm].contiguous().to(cuda), b[perm].to(cuda), nat.EPI_BF16_LN_BLK, q_bk, ln_rs=rs,
                    ln_c=c[perm].to(cuda))
    torch.cuda.synchronize()
    assert torch.equal(q_bk, nat.to_row_blocked(q_rm))
    kp = (torch.rand(M, generator=g) < 0.3).float().to(cuda) if masked else None
    o_rm = nat.op_attention(q_rm, frames, 256, NH, 50.0, key_pad=kp)
    o_bk = torch.empty_like(o_rm)
    nat.call("vp_dev_attention_spatial_blk", q_bk.data_ptr(), o_bk.data_ptr(), frames, NH, 50.0,
             kp.data_ptr() if kp is not None else None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(o_rm, o_bk)


@pytest.mark.parametrize("padded", [False, True])
@pytest.mark.parametrize("M,D,F", [(2048, 768, 3072), (512, 1024, 4096)])
def test_ffn_pair_row_blocked_bitwise(cuda, padded, M, D, F):
    """The FFN pair over the row-blocked hidden activation (ffn_layer1 stores from the accumulator
    layout with W1's rows permuted, ffn_layer2 stages A from the blocks) is bitwise the row-major
    pair: the hidden activation is the row-major one re-laid, the output and its row statistics equal."""
    g = torch.Generator(device="cpu").manual_seed(M + F + padded)
    x = _bf(torch.randn(M, D, generator=g) * 2 + 0.5)
    w1 = _bf(torch.randn(F, D, generator=g) / D ** 0.5)
    b1 = torch.randn(F, generator=g) * 0.1
    c1 = w1.double().sum(1).float()
    w2 = _bf(torch.randn(D, F, generator=g) / F ** 0.5)
    b2 = torch.randn(D, generator=g) * 0.1
    pad = (torch.rand(M, generator=g) < 0.2).float().to(cuda) if padded else None
    rs = torch.empty(M, 2, device=cuda)
    xd = x.to(cuda)
    nat.dev_ln_stats(xd, M, D, rs, from_partials=False)
    perm = torch.from_numpy(nat.ffn1_blk_rows(F))
    r0 = torch.randn(M, D, generator=g).to(torch.bfloat16).to(cuda)
    h_rm = torch.empty(M, F, device=cuda, dtype=torch.bfloat16)
    h_bk = torch.empty_like(h_rm)
    nat.dev_gemm_ln(xd, w1.to(cuda), b1.to(cuda), nat.EPI_GELU_LN, h_rm, rowpad=pad, ln_rs=rs, ln_c=c1.to(cuda))
    nat.dev_gemm_ln(xd, w1[perm].contiguous().to(cuda), b1[perm].to(cuda), nat.EPI_GELU_LN_BLK, h_bk, rowpad=pad,
                    ln_rs=rs, ln_c=c1[perm].to(cuda))
    torch.cuda.synchronize()
    assert torch.equal(h_bk, nat.to_row_blocked(h_rm))
    y_rm, y_bk = r0.clone(), r0.clone()
    st_rm = torch.empty(D // 128, M, 2, device=cuda)
    st_bk = torch.empty_like(st_rm)
    nat.dev_gemm_ln(h_rm, w2.to(cuda), b2.to(cuda), nat.EPI_RESID_FFN_BF16_ST, y_rm, resid=y_rm, rowpad=pad,
                    st_part=st_rm)
    nat.dev_gemm_ln(h_bk, w2.to(cuda), b2.to(cuda), nat.EPI_RESID_FFN_BF16_ST_BLK, y_bk, resid=y_bk, rowpad=pad,
                    st_part=st_bk)
    z_rm, z_bk = r0.clone(), r0.clone()
    nat.dev_gemm_kernel(4, h_rm, w2.to(cuda), b2.to(cuda), nat.EPI_RESID_FFN_BF16, z_rm, resid=z_rm, rowpad=pad)
    nat.dev_gemm_ln(h_bk, w2.to(cuda), b2.to(cuda), nat.EPI_RESID_FFN_BF16_BLK, z_bk, resid=z_bk, rowpad=pad)
    torch.cuda.synchronize()
    assert torch.equal(y_rm, y_bk) and torch.equal(st_rm, st_bk)
    assert torch.equal(z_rm, z_bk)


@pytest.mark.parametrize("epi", [nat.EPI_BF16_LN, nat.EPI_GELU_LN])
@pytest.mark.parametrize("M,N,K", [(1024, 2304, 768), (512, 3072, 768), (256, 1024, 1024)])
def test_gemm_ln_fold(cuda, epi, M, N, K):
    """LN(x).W + b computed as rstd*(x.W') - mean*rstd*c + b' with W' = W diag(gamma),
    b' = b + W.beta, c = row sums of bf16(W') -- against LN then GEMM in fp64 on the same bf16
    x.  The fold skips the reference's bf16 rounding of LN(x), so the bound is the bf16
    rounding of W' and of the output (rtol 2^-7) plus 2e-3 abs."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    x = _bf(torch.randn(M, K, generator=g) * 2 + 0.5)          # mean offset: exercises -mean*c
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g) * 0.1
    gam = 1 + torch.randn(K, generator=g) * 0.1
    bet = torch.randn(K, generator=g) * 0.1
    pad = (torch.rand(M, generator=g) < 0.2).float()
    wp = _bf(w * gam)
    c = wp.double().sum(1).float()
    bp = (b.double() + w.double() @ bet.double()).float()
    rs = torch.empty(M, 2, device=cuda)
    nat.dev_ln_stats(x.to(cuda), M, K, rs, from_partials=False)
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    nat.dev_gemm_ln(x.to(cuda), wp.to(cuda), bp.to(cuda), epi, out, ln_rs=rs, ln_c=c.to(cuda),
                    rowpad=pad.to(cuda) if epi == nat.EPI_GELU_LN else None)
    torch.cuda.synchronize()
    # (1) the kernel's arithmetic: the folded form with the bf16 W' it is given, in fp64
    xd = x.double()
    mu, var = xd.mean(1, keepdim=True), xd.var(1, unbiased=False, keepdim=True)
    rstd = 1 / torch.sqrt(var + 1e-6)
    y = rstd * (xd @ wp.double().T - mu * c.double()) + bp.double()
    # (2) the algebra: LayerNorm then GEMM with the unrounded weights (bf16 W' differs from W
    # by one rounding, so this bound is looser)
    y2 = _ln_ref(xd, gam.double(), bet.double()) @ w.double().T + b.double()
    if epi == nat.EPI_GELU_LN:
        keep = (1 - pad.double())[:, None]
        y = 0.5 * y * (1 + torch.erf(y / 2 ** 0.5)) * keep
        y2 = 0.5 * y2 * (1 + torch.erf(y2 / 2 ** 0.5)) * keep
    o = out.cpu().double()
    err = (o - y).abs()
    assert bool((err <= 2 ** -8 * y.abs() + 1e-4).all()), float(err.max())
    err2 = (o - y2).abs()
    assert float(err2.mean()) <= 2e-3 and float(err2.max()) <= 5e-2, (float(err2.mean()), float(err2.max()))


@pytest.mark.parametrize("epi", [nat.EPI_RESID_BF16_ST, nat.EPI_RESID_FFN_BF16_ST, nat.EPI_POS_BF16_ST])
def test_gemm_row_stats(cuda, epi):
    """A residual-stream producer's partial row statistics, finalised, equal the two-pass
    statistics of the bf16 rows it stored (ln_row_stats), and its stored values equal the
    plain epilogue's bit for bit."""
    M, N, K = 2048, 768, 768
    g = torch.Generator(device="cpu").manual_seed(epi)
    a = _bf(torch.randn(M, K, generator=g)).to(cuda)
    w = _bf(torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    x0 = (torch.randn(M, N, generator=g) * 3 + 1).to(cuda).to(torch.bfloat16)
    pos = torch.randn(256, N, generator=g).to(cuda) if epi == nat.EPI_POS_BF16_ST else None
    resid = epi != nat.EPI_POS_BF16_ST
    plain = {nat.EPI_RESID_BF16_ST: nat.EPI_RESID_BF16, nat.EPI_RESID_FFN_BF16_ST: nat.EPI_RESID_FFN_BF16,
             nat.EPI_POS_BF16_ST: nat.EPI_POS_BF16}[epi]
    o_st = x0.clone() if resid else torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    part = torch.full((N // 128, M, 2), float("nan"), device=cuda)
    nat.dev_gemm_ln(a, w, b, epi, o_st, resid=o_st if resid else None, pos=pos, st_part=part)
    o_pl = x0.clone() if resid else torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    nat.dev_gemm_kernel(4, a, w, b, plain, o_pl, resid=o_pl if resid else None, pos=pos)
    rs_p = torch.empty(M, 2, device=cuda)
    rs_r = torch.empty(M, 2, device=cuda)
    nat.dev_ln_stats(part, M, N, rs_p, from_partials=True)
    nat.dev_ln_stats(o_st, M, N, rs_r, from_partials=False)
    torch.cuda.synchronize()
    assert torch.equal(o_st, o_pl)
    xd = o_st.double()
    mean, var = xd.mean(1), xd.var(1, unbiased=False)
    rstd = 1 / torch.sqrt(var + 1e-6)
    ref = torch.stack([rstd, -mean * rstd], 1)
    assert torch.allclose(rs_p.double(), ref, rtol=2e-5, atol=1e-5)
    assert torch.allclose(rs_r.double(), ref, rtol=2e-5, atol=1e-5)



@pytest.mark.parametrize("heads", [12, 16])
def test_temporal_attention_fused_kernels_vs_unfused(cuda, heads):
    """The two fused temporal-attention launches (EPI_QK_TATTN_LN -> P, EPI_V_TATTN_LN -> O) on one
    layer with many GEMM tiles (M = 8192 rows = 512 sequences of T = 16; Base and Large head counts)
    against the unfused pair on the same inputs: the LN-folded q|k|v GEMM (EPI_BF16_LN) then the
    temporal attention kernel.  q, k, v are the same bf16 values on both paths; the fused path
    rounds the normalised probabilities to bf16 (the reference's probs.astype(fprop)), the unfused
    kernel the unnormalised numerators, so per element |O_f - O_u| <= 2^-6 |O_u| + 2^-7 max|v| of the
    (sequence, head) -- a few bf16 ulps -- with the mean far below.  Also against fp64 attention on
    the unfused path's bf16 q|k|v."""
    D = heads * 64
    M, S = 8192, 16
    nseq = M // S
    g = torch.Generator(device="cpu").manual_seed(heads)
    x = _bf(torch.randn(M, D, generator=g) * 2 + 0.3)
    w = torch.randn(3 * D, D, generator=g) / D ** 0.5
    w[:D] *= 0.125 * 4  # q rows carry the folded dh^-0.5 (with some extra spread of the logits)
    wp = _bf(w)
    b = (torch.randn(3 * D, generator=g) * 0.1).float()
    c = wp.double().sum(1).float()
    xc, wpc, bc, cc = x.to(cuda), wp.to(cuda), b.to(cuda), c.to(cuda)
    rs = torch.empty(M, 2, device=cuda)
    nat.dev_ln_stats(xc, M, D, rs, from_partials=False)
    # unfused: q|k|v (bf16) then the temporal kernel
    qkv = torch.empty(M, 3 * D, device=cuda, dtype=torch.bfloat16)
    nat.dev_gemm_ln(xc, wpc, bc, nat.EPI_BF16_LN, qkv, ln_rs=rs, ln_c=cc)
    o_u = nat.op_attention(qkv, nseq, S, heads, 50.0)
    # fused: [q_h | k_h] rows per head, then the v rows
    perm = torch.cat([torch.cat([torch.arange(h * 64, h * 64 + 64), D + torch.arange(h * 64, h * 64 + 64)])
                      for h in range(heads)])
    wqk, bqk, cqk = wpc[perm.to(cuda)].contiguous(), bc[perm.to(cuda)].contiguous(), cc[perm.to(cuda)].contiguous()
    p = torch.empty(nseq * heads * 256, device=cuda, dtype=torch.bfloat16)
    nat.dev_gemm_tattn(0, xc, wqk, bqk, rs, cqk, p, heads, 50.0)
    o_f = torch.empty(M, D, device=cuda, dtype=torch.bfloat16)
    nat.dev_gemm_tattn(1, xc, wpc[2 * D:].contiguous(), bc[2 * D:].contiguous(), rs, cc[2 * D:].contiguous(), o_f,
                       heads, 50.0, p=p)
    torch.cuda.synchronize()
    q = qkv.double().cpu().reshape(nseq, S, 3, heads, 64)
    qh, kh, vh = q[:, :, 0], q[:, :, 1], q[:, :, 2]                       # [nseq, S, heads, 64]
    logits = torch.einsum("nqhd,nkhd->nhqk", qh, kh)
    logits = 50.0 * torch.tanh(logits / 50.0)
    ref = torch.einsum("nhqk,nkhd->nqhd", torch.softmax(logits, -1), vh).reshape(M, D)
    vmax = vh.abs().amax(dim=(1, 3), keepdim=True).expand(nseq, S, heads, 64).reshape(M, D)
    of, ou = o_f.double().cpu(), o_u.double().cpu()
    d = (of - ou).abs()
    bound = 2 ** -6 * ou.abs() + 2 ** -7 * vmax
    print(f"heads {heads}: fused vs unfused max {float(d.max()):.3e} mean {float(d.mean()):.3e}; vs fp64 "
          f"fused {float((of - ref).abs().max()):.3e} unfused {float((ou - ref).abs().max()):.3e}")
    assert bool((d <= bound).all()), float((d - bound).max())
    assert float(d.mean()) <= 2e-3 * float(ou.abs().mean()) + 1e-4
    for o in (of, ou):
        assert bool(((o - ref).abs() <= 2 ** -7 * ref.abs() + 2 ** -7 * vmax).all())


@pytest.mark.parametrize("frames,P", [(3, 18), (9, 18), (3, 16), (3, 14), (4, 10), (5, 4)])
def test_patch_embed_fused_from_frames(cuda, frames, P):
    """The fused patch embedding (gemm_bf16_w4_video: the GEMM stages its A tiles straight from the
    bf16 frames in 16-B chunks of the patch pixel rows, no patch tensor) against the two-kernel
    path (patchify -> [M, 1024] patches -> GEMM) and against fp64 on the same bf16 frames: the sums
    differ only in their fp32 order (at most one bf16 ulp apart), and the fused result is within one
    bf16 rounding of fp64.  The chunk that overlaps its predecessor must meet zero weights there.
    Every even P the fused path takes (vp_kernels.h video_patch_ok): 3P = 54, 48, 42, 30, 12 values
    per pixel row, i.e. 7 / 6 / 6 / 4 / 2 chunks with and without an overlapping last chunk."""
    D = 768
    g = torch.Generator(device="cpu").manual_seed(frames)
    v = _bf(torch.rand(frames, 16 * P, 16 * P, 3, generator=g) * 4 - 1)
    k = torch.randn(P * P * 3, D, generator=g) / (P * P * 3) ** 0.5
    kb = _bf(k)
    b = torch.randn(D, generator=g) * 0.1
    pos = torch.randn(256, D, generator=g) * 0.1
    wv = nat.video_patch_w(kb, P)
    wk = torch.zeros(D, 1024)
    wk[:, :P * P * 3] = kb.T
    vd = v.to(cuda)
    fused = torch.empty(frames * 256, D, device=cuda, dtype=torch.bfloat16)
    nat.dev_patch_embed(vd, P, _bf(wv).to(cuda), b.to(cuda), pos.to(cuda), fused)
    patches = nat.op_patchify(vd, P, 1024, torch.bfloat16)
    two = nat.op_gemm(patches, _bf(wk).to(cuda), b.to(cuda), nat.EPI_POS_BF16, pos=pos.to(cuda))
    torch.cuda.synchronize()
    pt = orc.image_to_patch(v.double().numpy(), P).reshape(-1, P * P * 3)
    ref = pt @ kb.double().numpy() + b.double().numpy() + np.tile(pos.double().numpy(), (frames, 1))
    f, t = fused.double().cpu().numpy(), two.double().cpu().numpy()
    # two fp32 sums rounded to bf16 independently: at most one bf16 ulp apart (2^-7 relative just above
    # a power of two); each within half an ulp of fp64 plus the fp32 summation error
    assert np.all(np.abs(f - t) <= 2 ** -7 * np.abs(ref) + 1e-5), np.abs(f - t).max()
    assert np.all(np.abs(f - ref) <= 2 ** -8 * np.abs(ref) + 1e-4), np.abs(f - ref).max()
    print(f"fused patch embedding P={P}, {frames} frames: vs two-kernel max {np.abs(f - t).max():.3e} "
          f"(mean {np.abs(f - t).mean():.2e}); vs fp64 max {np.abs(f - ref).max():.3e}")


def test_patch_embed_fused_rejects_odd_patch(cuda):
    """Odd P would put the 16-B chunks at 2-B offsets in the frame: the fused launcher refuses them
    (the encoder takes patchify + GEMM for such grids, test_gpu_geometry.py)."""
    P, D = 9, 768
    v = torch.zeros(1, 16 * P, 16 * P, 3, device=cuda, dtype=torch.bfloat16)
    wv = torch.zeros(D, 64 * P, device=cuda, dtype=torch.bfloat16)
    out = torch.empty(256, D, device=cuda, dtype=torch.bfloat16)
    with pytest.raises(ValueError, match="even patch size"):
        nat.dev_patch_embed(v, P, wv, torch.zeros(D, device=cuda), torch.zeros(256, D, device=cuda), out)


@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (1024, 2304, 768), (384, 256, 3072), (1280, 640, 16)])
@pytest.mark.parametrize("epi", [nat.EPI_STORE, nat.EPI_GELU, nat.EPI_RESID, nat.EPI_POS, nat.EPI_RESID_FFN])
def test_gemm_f32_kernels(cuda, M, N, K, epi):
    """Both fp32 GEMM kernels (round 1's 16x16x4 one, which = 32, and the 32x32x2 product kernel, 33) on
    every fp32 epilogue, odd tile counts (XCD-contiguous ranges need a grid % 8 == 0) and a single K-tile,
    against fp64: exact fp32 products, fp32 sums in different orders, so each within 2e-5 of fp64."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    a = torch.randn(M, K, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    pad = (torch.rand(M, generator=g) < 0.25).float().to(cuda)
    x0 = torch.randn(M, N, generator=g).to(cuda)
    pos = torch.randn(256, N, generator=g).to(cuda) if epi == nat.EPI_POS else None
    y = a.double() @ w.double().T + b.double()
    keep = (1 - pad.double())[:, None]
    if epi == nat.EPI_GELU:
        ref = 0.5 * y * (1 + torch.erf(y / 2 ** 0.5)) * keep
    elif epi in (nat.EPI_RESID, nat.EPI_RESID_FFN):
        ref = x0.double() + y * keep
    elif epi == nat.EPI_POS:
        ref = y + pos.double().repeat(M // 256 + 1, 1)[:M]
    else:
        ref = y
    for which in (32, 33):
        o = x0.clone()
        nat.dev_gemm_kernel(which, a, w, b, epi, o, resid=o if epi in (nat.EPI_RESID, nat.EPI_RESID_FFN) else None,
                            pos=pos, rowpad=pad if epi != nat.EPI_POS and epi != nat.EPI_STORE else None)
        torch.cuda.synchronize()
        err = float((o.double() - ref).abs().max())
        assert err < 2e-5, (which, err)


@pytest.mark.parametrize("M,N,K,pad_a,pad_w", [(384, 256, 80, 12, 4), (256, 384, 768, 4, 36), (128, 128, 16, 0, 8)])
def test_gemm_f32_strided_operands(cuda, M, N, K, pad_a, pad_w):
    """The fp32 GEMM's LDS-DMA staging addresses A / W rows through lda / ldw (buffer descriptors over the tile's
    128 rows): row-strided operands (views of wider tensors, odd K-tile counts) against fp64, and the row
    strides it cannot stage (not a multiple of 4 floats, below K) refused with VP_EINVAL before any launch."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(M, K + pad_a, generator=g).to(cuda)
    Wt = (torch.randn(N, K + pad_w, generator=g) / K ** 0.5).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    a, w = A[:, :K], Wt[:, :K]
    assert a.stride(0) == K + pad_a and w.stride(0) == K + pad_w
    y = a.double() @ w.double().T + b.double()
    for epi in (nat.EPI_STORE, nat.EPI_GELU):
        out = nat.op_gemm(a, w, b, epi)
        torch.cuda.synchronize()
        ref = 0.5 * y * (1 + torch.erf(y / 2 ** 0.5)) if epi == nat.EPI_GELU else y
        err = float((out.double() - ref).abs().max())
        assert err < 2e-5, (epi, err)
    bad = torch.randn(M, K + 1, generator=g).to(cuda)[:, :K]  # lda = K + 1: rows not 16-B aligned
    with pytest.raises(ValueError, match="lda"):
        nat.op_gemm(bad, w, b, nat.EPI_STORE)
