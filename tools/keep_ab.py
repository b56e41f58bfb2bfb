"""A/B of the ffn_layer1 epilogue builds in one process: EPI_GELU_BF16_LN without padded rows
(rowpad = NULL -> the no-(1 - rowpad) build, DIAG 512) vs with an all-zero rowpad (the build that
multiplies by 1 - rowpad).  Interleaved rounds; outputs must be bitwise equal."""
import os
import sys

os.environ.setdefault("VP_DIAG_LIB", "1")  # ablation builds live in the diag library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]
import torch  # noqa: E402

from videoprism import _native as nat  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    M, N, K = 131072, 3072, 768
    g = torch.Generator(device=dev).manual_seed(0)
    a = (torch.rand((M, K), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand((N, K), generator=g, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    rs = torch.stack([torch.full((M,), 1.3, device=dev), torch.full((M,), -0.1, device=dev)], 1).contiguous()
    c = torch.rand(N, generator=g, device=dev)
    zero_pad = torch.zeros(M, device=dev)
    o1 = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    o2 = torch.empty_like(o1)
    f1 = lambda: nat.dev_gemm_ln(a, w, b, nat.EPI_GELU_LN, o1, ln_rs=rs, ln_c=c)  # noqa: E731
    f2 = lambda: nat.dev_gemm_ln(a, w, b, nat.EPI_GELU_LN, o2, rowpad=zero_pad, ln_rs=rs, ln_c=c)  # noqa: E731
    o3 = torch.empty_like(o1)
    f3 = lambda: nat.dev_gemm_ln(a, w, b, 3009, o3, ln_rs=rs, ln_c=c)  # noqa: E731
    o4 = torch.empty_like(o1)
    f4 = lambda: nat.dev_gemm_ln(a, w, b, 3010, o4, ln_rs=rs, ln_c=c)  # noqa: E731
    f1()
    f2()
    f3()
    f4()
    torch.cuda.synchronize()
    print("bitwise equal:", bool(torch.equal(o1, o2)), bool(torch.equal(o1, o3)), bool(torch.equal(o1, o4)))
    r1, r2, r3, r4 = [], [], [], []
    for _ in range(5):
        r1.append(timeit(f1))
        r2.append(timeit(f2))
        r3.append(timeit(f3))
        r4.append(timeit(f4))
    print(f"scalar GELU: {min(r4)*1e3:.1f} us")
    print(f"ffn1 GELU+LN epilogue: no-rowpad build {min(r1)*1e3:.1f} us   rowpad multiply (NULL) "
          f"{min(r3)*1e3:.1f} us   zero rowpad array {min(r2)*1e3:.1f} us")


if __name__ == "__main__":
    main()
