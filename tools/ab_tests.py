"""A/B equality checks of the tools' diag library (VP_DIAG_LIB=1; `make -C videoprism-mlx_amd diag`):
the overlapped-epilogue GEMM (gemm_bf16_ov) and the 8-wave GEMM with the 4-wave pipeline must be
bitwise equal to the production kernels.  Not part of tests/: the product library carries none of
these builds.  Run on the GPU box:  VP_DIAG_LIB=1 python tools/ab_tests.py"""
import os
import sys

os.environ["VP_DIAG_LIB"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from videoprism import _native as nat  # noqa: E402


def _bf(t):
    return t.to(torch.bfloat16)


def ov_vs_w4(M=16384, N=2304, K=768):
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = _bf(torch.randn(M, K, generator=g)).cuda()
    w = _bf(torch.randn(N, K, generator=g) / K ** 0.5).cuda()
    b = (torch.randn(N, generator=g) * 0.1).cuda()
    for epi in (nat.EPI_STORE, nat.EPI_GELU, nat.EPI_RESID_BF16):
        x0 = torch.randn(M, N, generator=g).cuda().to(torch.bfloat16)
        outs = {}
        for which in (4, 2):
            o = x0.clone() if epi == nat.EPI_RESID_BF16 else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            r = o if epi == nat.EPI_RESID_BF16 else None
            if which == 4:
                nat.dev_gemm_kernel(4, a, w, b, epi, o, resid=r)
            else:
                nat.dev_gemm_ov(a, w, b, epi, o, resid=r)
            outs[which] = o
        torch.cuda.synchronize()
        print(f"ov vs w4 epi {epi}: bitwise {torch.equal(outs[2], outs[4])}")


def w8b_vs_w4():
    """the 8-wave GEMM with the 4-wave pipeline (tools/diag/csrc/gemm_bf16_w8b.hip) against the
    4-wave kernel, EPI_BF16 and ffn_layer1's LN-fold + GELU epilogue (with / without padded rows)"""
    for M, N, K in ((4096, 3072, 768), (1280, 768, 704), (2048, 768, 3072)):
        g = torch.Generator(device="cpu").manual_seed(M + N + K)
        a = _bf(torch.randn(M, K, generator=g)).cuda()
        w = _bf(torch.randn(N, K, generator=g) / K ** 0.5).cuda()
        b = (torch.randn(N, generator=g) * 0.1).cuda()
        rs = torch.stack([torch.rand(M, generator=g) + 0.5, torch.randn(M, generator=g) * 0.3], 1).contiguous().cuda()
        c = torch.randn(N, generator=g).cuda()
        for epi, pad in ((nat.EPI_STORE, None), (nat.EPI_GELU_LN, None),
                         (nat.EPI_GELU_LN, (torch.rand(M, generator=g) < 0.2).float().cuda())):
            o4 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            o8 = torch.empty_like(o4)
            if epi == nat.EPI_STORE:
                nat.dev_gemm_kernel(4, a, w, b, epi, o4)
            else:
                nat.dev_gemm_ln(a, w, b, epi, o4, rowpad=pad, ln_rs=rs, ln_c=c)
            nat.dev_gemm_w8b(a, w, b, epi, o8, rowpad=pad, ln_rs=rs, ln_c=c)
            torch.cuda.synchronize()
            print(f"w8b vs w4 ({M}, {N}, {K}) epi {epi} rowpad {pad is not None}: bitwise {torch.equal(o4, o8)}")


if __name__ == "__main__":
    w8b_vs_w4()
    ov_vs_w4()
