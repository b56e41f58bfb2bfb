"""fp32 GEMM A/B (fprop_dtype=float32 path, gemm_f32.hip): round 1's v_mfma_f32_16x16x4_f32 kernel
(vp_dev_gemm_kernel which = 32) against the v_mfma_f32_32x32x2_f32 kernel (33) at the Base forward's shapes
(M = B * 16 * 256 rows), interleaved rounds in one process; both checked against fp64 on sampled rows."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]
import torch  # noqa: E402

from videoprism import _native as nat  # noqa: E402


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


VERS = (32, 33)


def main(B=4):
    dev = torch.device("cuda:0")
    M = B * 16 * 256
    shapes = {"qkv": (2304, 768, nat.EPI_STORE), "post": (768, 768, nat.EPI_RESID),
              "ffn1": (3072, 768, nat.EPI_GELU), "ffn2": (768, 3072, nat.EPI_RESID_FFN)}
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (N, K, epi) in shapes.items():
        a = torch.randn((M, K), generator=g, device=dev)
        w = torch.randn((N, K), generator=g, device=dev) / K ** 0.5
        b = torch.randn((N,), generator=g, device=dev) * 0.1
        x0 = torch.randn((M, N), generator=g, device=dev)
        outs = {v: x0.clone() for v in VERS}
        resid = epi in (nat.EPI_RESID, nat.EPI_RESID_FFN)
        fns = {v: (lambda v=v: nat.dev_gemm_kernel(v, a, w, b, epi, outs[v], resid=outs[v] if resid else None))
               for v in VERS}
        for v in VERS:  # one call each from the same x0 for the value check
            outs[v].copy_(x0)
            fns[v]()
        torch.cuda.synchronize()
        rows = torch.arange(0, M, 997, device=dev)
        y = a[rows].double() @ w.double().T + b.double()
        if epi == nat.EPI_GELU:
            y = 0.5 * y * (1 + torch.erf(y / 2 ** 0.5))
        if resid:
            y = y + x0[rows].double()
        err = {v: float((outs[v][rows].double() - y).abs().max()) for v in VERS}
        res = {v: [] for v in VERS}
        for _ in range(3):
            for v in VERS:
                res[v].append(timeit(fns[v]))
        flop = 2.0 * M * N * K
        print(f"{name} M={M} N={N} K={K}: " + "  ".join(
            f"v{v}: {min(res[v]) * 1e3:7.1f} us ({flop / min(res[v]) / 1e9:5.1f} TF, max-abs vs fp64 {err[v]:.2e})"
            for v in VERS), flush=True)


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:2]])
