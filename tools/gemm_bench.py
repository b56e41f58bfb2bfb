"""GEMM microbenchmark at the encoder's shapes: both HIP kernels (4-wave `gemm_bf16_w4`,
8-wave `gemm_bf16`) with the forward's epilogues, against torch.matmul (hipBLASLt) as a
known-good reference on the same device and data (no epilogue on the torch side).

  python tools/gemm_bench.py            # kernels vs torch, plus the w4 == w8 bitwise check
  python tools/gemm_bench.py ablate     # the 4-wave kernel's ablation builds (diag library: no
                                        # ds_reads / no staging loads / no epilogue), 2-stage and S3
  python tools/gemm_bench.py fold       # LN-folded / row-statistics epilogues vs the plain ones
  python tools/gemm_bench.py msize      # the FFN GEMMs at smaller M (Infinity-Cache resident A)
  python tools/gemm_bench.py tattn      # fused temporal attention launches vs their no-epilogue builds
(Rounds 1-4 experiments -- early loads, prefetch distances, start skew, tile orders, XCD pairs, plain
stores, the overlapped-epilogue and 8-wave/4-wave-pipeline kernels -- are recorded in
profiles/HISTORY.md with their numbers; their builds are in git history.)
"""
import ctypes
import os
import sys

os.environ.setdefault("VP_DIAG_LIB", "1")  # ablation builds live in the diag library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]
import torch  # noqa: E402

from videoprism import _native as nat  # noqa: E402

M_TOK = 131072  # B=32 clips x 16 frames x 256 patches
SHAPES = [  # name, M, N, K, epilogue (as in vp_forward's bf16 path)
    ("qkv", M_TOK, 2304, 768, nat.EPI_STORE),
    ("post", M_TOK, 768, 768, nat.EPI_RESID_BF16),
    ("ffn1", M_TOK, 3072, 768, nat.EPI_GELU),
    ("ffn2", M_TOK, 768, 3072, nat.EPI_RESID_FFN_BF16),
]
EXTRA = [("ffn1-noact", M_TOK, 3072, 768, nat.EPI_STORE)]  # prices the GELU epilogue


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


def operands(M, N, K, g, dev):
    a = (torch.rand((M, K), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand((N, K), generator=g, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    return a, w, b


def compare(dev, g):
    for name, M, N, K, epi in SHAPES + EXTRA:
        a, w, b = operands(M, N, K, g, dev)
        resid = epi in (nat.EPI_RESID_BF16, nat.EPI_RESID_FFN_BF16)
        x0 = torch.randn((M, N), generator=g, device=dev).to(torch.bfloat16) if resid else None
        outs = {}
        for which in (8, 4):
            o = x0.clone() if resid else torch.empty((M, N), device=dev, dtype=torch.bfloat16)
            nat.dev_gemm_kernel(which, a, w, b, epi, o, resid=o if resid else None)
            outs[which] = o
        torch.cuda.synchronize()
        same = bool(torch.equal(outs[4], outs[8]))
        del outs
        o = x0.clone() if resid else torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        fns = {"w8": lambda: nat.dev_gemm_kernel(8, a, w, b, epi, o, resid=o if resid else None),
               "w4": lambda: nat.dev_gemm_kernel(4, a, w, b, epi, o, resid=o if resid else None),
               "torch": lambda: torch.matmul(a, w.t())}
        res = {k: [] for k in fns}
        for _ in range(3):  # interleaved rounds
            for k, f in fns.items():
                res[k].append(timeit(f))
        flop = 2.0 * M * N * K
        print(f"{name:5s} M={M} N={N} K={K} epi={epi} w4==w8:{same}: " + " | ".join(
            f"{k} {min(v)*1e3:7.1f} us {flop/min(v)/1e9:7.1f} TF" for k, v in res.items()), flush=True)


def ablate(dev, g):
    """The product 4-wave kernel (EPI_BF16) and its ablation builds (diag library): abl 2 = no ds_reads
    in the K-loop, 4 = no staging loads, 6 = neither, 8 = no epilogue, 14 = none of the three; both
    the 2-stage and the S3 staging."""
    abls = [0, 2, 4, 6, 8, 14]
    for name, M, N, K, _ in SHAPES:
        a, w, b = operands(M, N, K, g, dev)
        o = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        for s3 in (False, True):
            res = {d: [] for d in abls}
            for _ in range(3):
                for d in abls:
                    res[d].append(timeit(lambda: nat.dev_gemm_w4_abl(a, w, b, o, d, s3=s3), iters=10, warm=2))
            flop = 2.0 * M * N * K
            print(f"{name} {'S3' if s3 else '2-stage'} ablations:", " ".join(f"a{d}:{flop/min(t)/1e9:6.1f}TF"
                                                                          for d, t in res.items()),
                  "| us:", " ".join(f"a{d}:{min(t)*1e3:6.1f}" for d, t in res.items()), flush=True)


def folded(dev, g):
    """The forward's LN-folded / row-statistics epilogues at the encoder shapes vs the plain ones."""
    cases = [("qkv", 2304, 768, nat.EPI_STORE, nat.EPI_BF16_LN), ("post", 768, 768, nat.EPI_RESID_BF16, nat.EPI_RESID_BF16_ST),
             ("ffn1", 3072, 768, nat.EPI_GELU, nat.EPI_GELU_LN), ("ffn2", 768, 3072, nat.EPI_RESID_FFN_BF16, nat.EPI_RESID_FFN_BF16_ST)]
    for name, N, K, plain, fold in cases:
        M = M_TOK
        a, w, b = operands(M, N, K, g, dev)
        o = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        resid = plain in (nat.EPI_RESID_BF16, nat.EPI_RESID_FFN_BF16)
        rs = torch.stack([torch.ones(M, device=dev), torch.zeros(M, device=dev)], 1).contiguous()
        c = torch.zeros(N, device=dev)
        part = torch.empty((N // 128, M, 2), device=dev)
        fns = {"plain": lambda: nat.dev_gemm_kernel(4, a, w, b, plain, o, resid=o if resid else None),
               "fold": lambda: nat.dev_gemm_ln(a, w, b, fold, o, resid=o if resid else None, ln_rs=rs, ln_c=c,
                                               st_part=part)}
        res = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                res[k].append(timeit(f))
        flop = 2.0 * M * N * K
        print(f"{name} epi {plain} vs {fold}: " + " | ".join(f"{k} {min(v)*1e3:7.1f} us {flop/min(v)/1e9:7.1f} TF"
                                                          for k, v in res.items()), flush=True)


def msize(dev, g):
    """ffn_layer2 / ffn_layer1 at smaller M (A resident in the 256 MiB Infinity Cache when it fits):
    per-FLOP rate vs the B=32 shape (forward epilogues, isolated back-to-back launches)."""
    for name, N, K, epi in (("ffn2", 768, 3072, nat.EPI_RESID_FFN_BF16_ST), ("ffn1", 3072, 768, nat.EPI_GELU_LN)):
        for M in (131072, 65536, 32768):
            a, w, b = operands(M, N, K, g, dev)
            rs = torch.stack([torch.ones(M, device=dev), torch.zeros(M, device=dev)], 1).contiguous()
            c = torch.zeros(N, device=dev)
            part = torch.empty((N // 128, M, 2), device=dev)
            o = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
            resid = epi == nat.EPI_RESID_FFN_BF16_ST
            f = lambda: nat.dev_gemm_ln(a, w, b, epi, o, resid=o if resid else None, ln_rs=rs, ln_c=c, st_part=part)
            t = min(timeit(f) for _ in range(3))
            print(f"{name} M={M}: {t*1e3:7.1f} us {2.0*M*N*K/t/1e9:7.1f} TF", flush=True)
            del a, o, part, rs


def tattn(dev, g):
    """The fused temporal attention launches at the bench shape (M = 131072, D = 768, 12 heads): product
    builds and their no-epilogue builds (diag ABL 8, prices the epilogues); interleaved rounds."""
    M, D, H = M_TOK, 768, 12
    x = (torch.rand((M, D), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand((3 * D, D), generator=g, device=dev) * 2 - 1) / D ** 0.5).to(torch.bfloat16)
    b = torch.zeros(3 * D, device=dev)
    c = torch.zeros(3 * D, device=dev)
    rs = torch.stack([torch.ones(M, device=dev), torch.zeros(M, device=dev)], 1).contiguous()
    p = torch.empty(M // 16 * H * 256, device=dev, dtype=torch.bfloat16)
    o = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    st = lambda: torch.cuda.current_stream().cuda_stream
    wv = w[2 * D:].contiguous()
    def qk(abl):
        nat.call("vp_dev_gemm_tattn_abl", 0, abl, x.data_ptr(), w.data_ptr(), M, D, p.data_ptr(), b.data_ptr(),
                 rs.data_ptr(), c.data_ptr(), None, H, 50.0, st())
    def vv(abl):
        nat.call("vp_dev_gemm_tattn_abl", 1, abl, x.data_ptr(), wv.data_ptr(), M, D, o.data_ptr(), b.data_ptr(),
                 rs.data_ptr(), c.data_ptr(), p.data_ptr(), H, 50.0, st())
    qk(0)
    fns = {"qk": lambda: qk(0), "qk-noepi": lambda: qk(8), "v": lambda: vv(0), "v-noepi": lambda: vv(8)}
    res = {k: [] for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            res[k].append(timeit(f))
    print("tattn:", " | ".join(f"{k} {min(v)*1e3:7.1f} us" for k, v in res.items()), flush=True)


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    mode = sys.argv[1] if len(sys.argv) > 1 else ""
    modes = {"fold": folded, "ablate": ablate, "msize": msize, "tattn": tattn}
    modes.get(mode, compare)(dev, g)


if __name__ == "__main__":
    main()
