"""ffn_layer1 (default) or ffn_layer2 (`ffn2`) at the bench shape (M = 131072, N = 3072, K = 768; the product launch
gemm_bf16_w4_kernel<16, true, false>: LN fold + GELU into the row-blocked hidden) against its ablation builds
(diag library): a8 = no epilogue (the K-loop alone), a2 = no ds_reads, a4 = no staging loads, a14 = all three.
Prices the epilogue the ping-pong GEMM would have to hide; run it under tools/pmc_passes.sh for
the MFMA-busy / VALU / LDS / VMEM counters of each build.

    VP_DIAG_LIB=1 python tools/ffn1_split.py [ffn2]
(ffn2: gemm_bf16_w4_kernel<17, false, true>, M = 131072, N = 768, K = 3072, A = the row-blocked hidden.)
"""
import os
import sys

os.environ.setdefault("VP_DIAG_LIB", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]
import torch  # noqa: E402

from videoprism import _native as nat  # noqa: E402


def ffn2():
    dev = torch.device("cuda:0")
    M, N, K = 131072, 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn((M, K), generator=g, device=dev).to(torch.bfloat16)  # as the row-blocked layout: same bytes
    w = (torch.randn((N, K), generator=g, device=dev) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g, device=dev) * 0.1
    x0 = torch.randn((M, N), generator=g, device=dev).to(torch.bfloat16)
    x = x0.clone()
    st = torch.empty((N // 128, M, 2), device=dev)
    s_ = torch.cuda.current_stream().cuda_stream
    fns = {abl: (lambda abl=abl: nat.call("vp_dev_gemm_ffn2_abl", abl, a.data_ptr(), w.data_ptr(), M, N, K,
                                          x.data_ptr(), b.data_ptr(), st.data_ptr(), s_))
           for abl in (0, 8, 2, 4, 14)}
    run(fns, 2.0 * M * N * K, "ffn2")


def run(fns, flop, tag):
    res = {k: [] for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            for _ in range(2):
                f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                f()
            e.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(e) / 10)
    names = {0: "product", 8: "no epilogue", 2: "no ds_reads", 4: "no staging", 14: "MFMAs only"}
    for k, v in res.items():
        t = min(v)
        print(f"{tag} a{k:<2d} {names[k]:12s}: {t * 1e3:7.1f} us  {flop / t / 1e9:7.1f} TF", flush=True)


def main():
    dev = torch.device("cuda:0")
    M, N, K = 131072, 3072, 768
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn((M, K), generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn((N, K), generator=g, device=dev) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g, device=dev) * 0.1
    c = w.float().sum(1).contiguous()
    rs = torch.stack([torch.rand(M, generator=g, device=dev) + 0.5, torch.randn(M, generator=g, device=dev)], 1)
    rs = rs.contiguous()
    o = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    fns = {abl: (lambda abl=abl: nat.call("vp_dev_gemm_ffn1_abl", abl, a.data_ptr(), w.data_ptr(), M, N, K,
                                          o.data_ptr(), b.data_ptr(), rs.data_ptr(), c.data_ptr(), st))
           for abl in (0, 8, 2, 4, 14)}
    run(fns, 2.0 * M * N * K, "ffn1")


if __name__ == "__main__":
    if sys.argv[1:2] == ["ffn2"]:
        ffn2()
    else:
        main()
