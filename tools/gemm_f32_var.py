"""fp32 GEMM schedule variants and ablations (tools/diag/csrc/gemm_f32_var.hip, diag library only) against
the product kernel (vp_dev_gemm_kernel which = 33) at the Base forward's fp32 shapes, interleaved rounds in
one process.  abl 0 variants must equal the product bitwise; ablations (2 = no LDS reads, 4 = no staging,
8 = no epilogue, 16 = no barrier) price the parts of the K-loop.
Usage (GPU): VP_DIAG_LIB=1 python tools/gemm_f32_var.py [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]
os.environ.setdefault("VP_DIAG_LIB", "1")
import torch  # noqa: E402

from videoprism import _native as nat  # noqa: E402

CASES = [(0, 0), (3, 64), (8, 0), (9, 6)]


def timeit(fn, iters=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main(B=8):
    dev = torch.device("cuda:0")
    M = B * 16 * 256
    shapes = {"qkv": (2304, 768, 0), "ffn1": (3072, 768, 1), "post": (768, 768, 0), "ffn2": (768, 3072, 0)}
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (N, K, gelu) in shapes.items():
        a = torch.randn((M, K), generator=g, device=dev)
        w = torch.randn((N, K), generator=g, device=dev) / K ** 0.5
        b = torch.randn((N,), generator=g, device=dev) * 0.1
        prod = torch.empty((M, N), device=dev)
        outs = {c: torch.empty((M, N), device=dev) for c in CASES}
        epi_p = nat.EPI_GELU if gelu else nat.EPI_STORE

        def fprod():
            nat.dev_gemm_kernel(33, a, w, b, epi_p, prod)

        def fvar(c):
            nat.call("vp_dev_gemm_f32_var", c[0], c[1], gelu, nat._ptr(a), nat._ptr(w), M, N, K,
                     nat._ptr(outs[c]), nat._ptr(b), nat._stream(None))

        fns = {"prod": fprod}
        fns.update({f"v{c[0]}a{c[1]}": (lambda c=c: fvar(c)) for c in CASES})
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        same = {c: bool(torch.equal(outs[c], prod)) for c in CASES if c[1] == 0 and c[0] < 5}
        ref_pers = outs[(3, 64)] if gelu else prod  # the persistent / reordered kernels use the packed GELU
        for c in CASES:
            if c[0] >= 5:
                same[c] = bool(torch.equal(outs[c], ref_pers))
        if gelu:  # the libm-free GELU (abl 32) against fp64 on sampled rows, beside the product's
            rows = torch.arange(0, M, 97, device=dev)
            y = a[rows].double() @ w.double().T + b.double()
            y = 0.5 * y * (1 + torch.erf(y / 2 ** 0.5))
            for c in [("prod", prod)] + [(c, outs[c]) for c in CASES if c[1] in (0, 64) or c[0] >= 5]:
                d = (c[1][rows].double() - y).abs()
                print(f"  {str(c[0]):8s} vs fp64: max {float(d.max()):.3e} mean {float(d.mean()):.3e}", flush=True)
        res = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                res[k].append(timeit(f))
        flop = 2.0 * M * N * K
        print(f"{name} M={M} N={N} K={K} (abl-0 variants bitwise equal to the product: {same})", flush=True)
        for k in fns:
            t = min(res[k])
            print(f"  {k:8s} {t * 1e3:8.1f} us  {flop / t / 1e9:6.1f} TF", flush=True)


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:2]])
