"""Times torch.matmul (hipBLASLt) at the encoder's GEMM shapes; run under rocprofv3 --kernel-trace
to see which library kernel (macro tile, MFMA shape) the vendor picks for each shape."""
import torch

M = 131072
dev = torch.device("cuda:0")
for N, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    for _ in range(5):
        torch.matmul(a, w.t())
    torch.cuda.synchronize()
    print(N, K, flush=True)
