"""Fused q|k|v projection + spatial attention (qkv_attention.hip) vs the unfused pair
(gemm_bf16_w4 EPI_BF16_LN -> q|k|v tensor -> attn_spatial_kernel) at the encoder's shape
(B=32 clips x 16 frames = 512 frames, D = 768, 12 heads).  Interleaved rounds, one process.

  python tools/qa_bench.py [frames]
"""
import os
import sys

os.environ.setdefault("VP_DIAG_LIB", "1")  # the fused kernel lives in the diag library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]
import torch  # noqa: E402

from videoprism import _native as nat  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dev = torch.device("cuda:0")
    heads, D, M = 12, 768, frames * 256
    mode = sys.argv[2] if len(sys.argv) > 2 else "dev"
    if mode == "cpu":  # the GPU test's generation (CPU generator, then copied)
        g = torch.Generator(device="cpu").manual_seed(100 + frames)
        x = torch.randn(M, D, generator=g).to(torch.bfloat16).to(dev)
        w = (torch.randn(3 * D, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(dev)
        b = (torch.randn(3 * D, generator=g) * 0.1).to(dev)
        c = torch.randn(3 * D, generator=g).to(dev)
        rs = torch.stack([torch.rand(M, generator=g) + 0.5, torch.randn(M, generator=g) * 0.1], 1).contiguous().to(dev)
    else:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(M, D, generator=g, device=dev).to(torch.bfloat16)
        w = (torch.randn(3 * D, D, generator=g, device=dev) / D ** 0.5).to(torch.bfloat16)
        b = torch.randn(3 * D, generator=g, device=dev) * 0.1
        c = torch.randn(3 * D, generator=g, device=dev)
        rs = torch.stack([torch.rand(M, generator=g, device=dev) + 0.5,
                          torch.randn(M, generator=g, device=dev) * 0.1], 1).contiguous()
        if mode == "ident":
            b.zero_(); c.zero_(); rs[:, 0] = 1.0; rs[:, 1] = 0.0
    qkv = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)
    o1 = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    o2 = torch.empty_like(o1)

    def unfused():
        nat.dev_gemm_ln(x, w, b, nat.EPI_BF16_LN, qkv, ln_rs=rs, ln_c=c)
        nat.op_attention(qkv, frames, 256, heads, 50.0, out=o1)

    def gemm_only():
        nat.dev_gemm_ln(x, w, b, nat.EPI_BF16_LN, qkv, ln_rs=rs, ln_c=c)

    def attn_only():
        nat.op_attention(qkv, frames, 256, heads, 50.0, out=o1)

    def fused():
        nat.dev_qkv_attention(x, rs, w, b, c, o2, frames, heads, 50.0)

    unfused()
    fused()
    torch.cuda.synchronize()
    o3 = o2.clone()
    fused()
    torch.cuda.synchronize()
    print("fused deterministic:", bool(torch.equal(o2, o3)), flush=True)
    print("bitwise equal:", bool(torch.equal(o1, o2)), flush=True)
    if not torch.equal(o1, o2):
        d = (o1.float() - o2.float()).abs().view(frames, 256, heads, 64)
        bad = (d > 0).any(dim=3).any(dim=1)  # [frames, heads]
        items = bad.nonzero().tolist()
        print(f"max abs diff {float(d.max()):.4g}; mismatching (frame, head) items: {len(items)} of "
              f"{frames * heads}; first: {items[:12]}", flush=True)
        per_tok = (d > 0).any(dim=3).float().sum(dim=1)  # tokens per (frame, head)
        print("mismatching tokens per bad item:", per_tok[bad][:12].tolist(), flush=True)
        f0, h0 = items[0]
        got = o2.view(frames, 256, heads, 64)[f0, :, h0]
        O1 = o1.view(frames, 256, heads, 64)
        print("got[0,:8]", got[0, :8].tolist(), "ref", O1[f0, 0, h0, :8].tolist(), flush=True)
    fns = {"unfused": unfused, "gemm_qkv": gemm_only, "attention": attn_only, "fused": fused,
           "fused_no_attn": lambda: nat.dev_qkv_attention(x, rs, w, b, c, o2, frames, heads, -1001.0),
           "fused_no_gemm": lambda: nat.dev_qkv_attention(x, rs, w, b, c, o2, frames, heads, -1002.0),
           "fused_neither": lambda: nat.dev_qkv_attention(x, rs, w, b, c, o2, frames, heads, -1003.0)}
    res = {k: [] for k in fns}
    for _ in range(5):
        for k, f in fns.items():
            res[k].append(timeit(f, iters=10, warm=2))
    gf = 2.0 * M * D * 3 * D + 4.0 * frames * 256 * 256 * D
    for k, v in res.items():
        t = min(v)
        print(f"{k:10s} {t*1e3:8.1f} us" + (f"  {gf / t / 1e9:7.1f} TFLOP/s (qkv GEMM + attention FLOPs)"
                                            if k in ("unfused", "fused") else ""), flush=True)


if __name__ == "__main__":
    main()
