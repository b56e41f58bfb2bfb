"""GEMM microbenchmark at the encoder's shapes: our HIP kernel (vp_op_gemm) vs
torch.matmul (hipBLASLt) as a known-good reference on the same device and data."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]
import torch  # noqa: E402

from videoprism import _native as nat  # noqa: E402

SHAPES = [  # name, M, N, K, epilogue
    ("qkv", 131072, 2304, 768, nat.EPI_STORE),
    ("post", 131072, 768, 768, nat.EPI_RESID),
    ("ffn1", 131072, 3072, 768, nat.EPI_GELU),
    ("ffn2", 131072, 768, 3072, nat.EPI_RESID_FFN),
]


def timeit(fn, iters=20, warm=3):
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


def variants(dev, g):
    import ctypes
    lib = nat.load()
    fn = lib.vp_dev_gemm_diag
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                   ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    for name, M, N, K, _ in SHAPES:
        a = (torch.rand((M, K), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand((N, K), generator=g, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        b = torch.zeros(N, device=dev)
        o = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        s = torch.cuda.current_stream().cuda_stream
        res = {v: [] for v in (0, 1, 8, 2, 10, 3)}
        for rnd in range(3):  # interleaved rounds (rule 24)
            for v in res:
                f = lambda: nat.check(fn(v, a.data_ptr(), w.data_ptr(), M, N, K, o.data_ptr(), b.data_ptr(), s))
                res[v].append(timeit(f, iters=10, warm=2))
        flop = 2.0 * M * N * K
        print(name, "diag", " ".join(f"d{v}:{flop/min(t)/1e9:6.1f}TF" for v, t in res.items()), flush=True)


def main():
    only = sys.argv[1:]
    if only == ["variants"]:
        variants(torch.device("cuda:0"), torch.Generator(device="cuda:0").manual_seed(0))
        return
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, N, K, epi in SHAPES:
        if only and name not in only:
            continue
        a = (torch.rand((M, K), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand((N, K), generator=g, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        b = torch.zeros(N, device=dev)
        x = torch.zeros((M, N), device=dev)
        o = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        flop = 2.0 * M * N * K
        if epi in (nat.EPI_RESID, nat.EPI_RESID_FFN):
            f = lambda: nat.op_gemm(a, w, b, epi, out=x, resid=x)
        else:
            f = lambda: nat.op_gemm(a, w, b, epi, out=o)
        import ctypes
        lib = nat.load()
        w4 = lib.vp_dev_gemm_w4
        w4.restype = ctypes.c_int
        w4.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                       ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        st = torch.cuda.current_stream().cuda_stream
        outp = x if epi in (nat.EPI_RESID, nat.EPI_RESID_FFN) else o
        g4 = lambda: nat.check(w4(epi, a.data_ptr(), w.data_ptr(), M, N, K, outp.data_ptr(), b.data_ptr(), x.data_ptr(), st))
        if epi in (nat.EPI_STORE, nat.EPI_GELU):
            ref_o = nat.op_gemm(a, w, b, epi, out=torch.empty_like(o)).float()
            g4(); torch.cuda.synchronize()
            print(f"  w4 vs w8 max|diff| {float((o.float() - ref_o).abs().max()):.3e}")
        res = {"w8": [], "w4": [], "torch": []}
        for _ in range(3):
            res["w8"].append(timeit(f))
            res["w4"].append(timeit(g4))
            res["torch"].append(timeit(lambda: torch.matmul(a, w.t())))
        print(f"{name:5s} M={M} N={N} K={K}: " + " | ".join(
            f"{k} {min(v)*1e3:7.1f} us {flop/min(v)/1e9:7.1f} TF" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
