"""GEMM microbenchmark at the encoder's shapes: both HIP kernels (4-wave `gemm_bf16_w4`,
8-wave `gemm_bf16`) with the forward's epilogues, against torch.matmul (hipBLASLt) as a
known-good reference on the same device and data (no epilogue on the torch side).

  python tools/gemm_bench.py            # kernels vs torch, plus w4 == w8 bitwise check
  python tools/gemm_bench.py w4var      # 4-wave ablation builds (DIAG bits, see the kernel)
  python tools/gemm_bench.py w8var      # 8-wave ablation builds
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
        o2 = x0.clone() if resid else torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        nat.dev_gemm_kernel(2, a, w, b, epi, o2, resid=o2 if resid else None)
        o4 = x0.clone() if resid else torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        nat.dev_gemm_kernel(4, a, w, b, epi, o4, resid=o4 if resid else None)
        same_ov = bool(torch.equal(o2, o4))
        del o2, o4
        fns = {"w8": lambda: nat.dev_gemm_kernel(8, a, w, b, epi, o, resid=o if resid else None),
               "w4": lambda: nat.dev_gemm_kernel(4, a, w, b, epi, o, resid=o if resid else None),
               "ov": lambda: nat.dev_gemm_kernel(2, a, w, b, epi, o, resid=o if resid else None),
               "torch": lambda: torch.matmul(a, w.t())}
        res = {k: [] for k in fns}
        for _ in range(3):  # interleaved rounds
            for k, f in fns.items():
                res[k].append(timeit(f))
        flop = 2.0 * M * N * K
        print(f"{name:5s} M={M} N={N} K={K} epi={epi} w4==w8:{same} ov==w4:{same_ov}: " + " | ".join(
            f"{k} {min(v)*1e3:7.1f} us {flop/min(v)/1e9:7.1f} TF" for k, v in res.items()), flush=True)


def variants(dev, g, which, diags):
    for name, M, N, K, _ in SHAPES:
        a, w, b = operands(M, N, K, g, dev)
        o = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        st = torch.cuda.current_stream().cuda_stream
        res = {d: [] for d in diags}
        for _ in range(3):
            for d in diags:
                if which in (2, 4):
                    f = lambda: nat.dev_gemm_kernel(which, a, w, b, (1000 + d) if d else 0, o)
                else:
                    lib = nat.load()
                    fn = lib.vp_dev_gemm_diag
                    fn.restype = ctypes.c_int
                    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                   ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p]
                    f = lambda: nat.check(fn(d, a.data_ptr(), w.data_ptr(), M, N, K, o.data_ptr(),
                                             b.data_ptr(), st))
                res[d].append(timeit(f, iters=10, warm=2))
        flop = 2.0 * M * N * K
        print(f"{name} w{which} ablations:", " ".join(f"d{d}:{flop/min(t)/1e9:6.1f}TF" for d, t in res.items()),
              "| us:", " ".join(f"d{d}:{min(t)*1e3:6.1f}" for d, t in res.items()), flush=True)


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


def skew(dev, g):
    """Start skew (DIAG 64, EPI_BF16): workgroup group (b>>3) % G of every XCD delays its first
    K-tile by group * d, so the CUs' epilogue store bursts stop coinciding (G, d swept)."""
    cfgs = [(1, 0), (2, 400), (2, 800), (2, 1200), (4, 300), (4, 600), (8, 150), (8, 300)]
    for name, M, N, K, _ in SHAPES:
        a, w, b = operands(M, N, K, g, dev)
        o = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        res = {c: [] for c in [None] + cfgs}
        for _ in range(3):
            for c in res:
                if c is None:
                    f = lambda: nat.dev_gemm_kernel(4, a, w, b, 0, o)
                else:
                    pos = torch.empty(c[0] * 10000 + c[1], device=dev)
                    f = lambda: nat.dev_gemm_kernel(4, a, w, b, 1064, o, pos=pos)
                res[c].append(timeit(f, iters=10, warm=2))
        print(f"{name} skew (G, d x10ns):", " ".join(f"{c}:{min(t)*1e3:6.1f}" for c, t in res.items()), flush=True)


def grouped(dev, g):
    """ffn_layer1 (production LN-folded GELU epilogue) with the N-tile grouped tile order
    (w4_ngrp) vs the ungrouped one (diag 3011) and the XCD-pair split of W (diag 3013), M = 131072
    and the Large shape."""
    for name, M, N, K in (("ffn1-base", M_TOK, 3072, 768), ("ffn1-large", 65536, 4096, 1024),
                          ("qkv-large", 65536, 3072, 1024)):
        a, w, b = operands(M, N, K, g, dev)
        o = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        rs = torch.stack([torch.ones(M, device=dev), torch.zeros(M, device=dev)], 1).contiguous()
        c = torch.zeros(N, device=dev)
        epi = nat.EPI_GELU_LN if name.startswith("ffn1") else nat.EPI_BF16_LN
        fns = {"grouped": lambda: nat.dev_gemm_ln(a, w, b, epi, o, ln_rs=rs, ln_c=c)}
        if epi == nat.EPI_GELU_LN:
            fns["ungrouped"] = lambda: nat.dev_gemm_ln(a, w, b, 3011, o, ln_rs=rs, ln_c=c)
            # XCD pairs: each XCD of a pair sweeps the pair's M-blocks over half of W (L2-resident)
            fns["xcd-pairs"] = lambda: nat.dev_gemm_ln(a, w, b, 3013, o, ln_rs=rs, ln_c=c)
            o2 = torch.empty_like(o)
            nat.dev_gemm_ln(a, w, b, epi, o, ln_rs=rs, ln_c=c)
            nat.dev_gemm_ln(a, w, b, 3013, o2, ln_rs=rs, ln_c=c)
            torch.cuda.synchronize()
            print(f"{name}: xcd-pairs == grouped (bitwise):", bool(torch.equal(o, o2)), flush=True)
            del o2
        res = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                res[k].append(timeit(f))
        flop = 2.0 * M * N * K
        print(f"{name}: " + " | ".join(f"{k} {min(v)*1e3:7.1f} us {flop/min(v)/1e9:7.1f} TF" for k, v in res.items()),
              flush=True)
        del a, o


def grouped_pmc(dev, g):
    """The three ffn_layer1 tile orders of `grouped`, 5 launches each and no timing loop, for
    rocprofv3 --pmc (one kernel symbol per order: FETCH_SIZE per launch is the A/W re-read)."""
    for name, M, N, K in (("ffn1-base", M_TOK, 3072, 768), ("ffn1-large", 65536, 4096, 1024)):
        a, w, b = operands(M, N, K, g, dev)
        o = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        rs = torch.stack([torch.ones(M, device=dev), torch.zeros(M, device=dev)], 1).contiguous()
        c = torch.zeros(N, device=dev)
        for code in (nat.EPI_GELU_LN, 3011, 3013):
            for _ in range(5):
                nat.dev_gemm_ln(a, w, b, code, o, ln_rs=rs, ln_c=c)
            torch.cuda.synchronize()
        print(f"{name}: done", flush=True)
        del a, o


def s3_ab(dev, g):
    """ffn_layer2 shape: S3 staging (production for K >= 2048: three A buffers, A pieces in h0)
    vs the PF 2 build it replaced -- plain epilogue, no epilogue, and the production residual +
    row-statistics epilogue."""
    M, N, K = M_TOK, 768, 3072
    a, w, b = operands(M, N, K, g, dev)
    o = torch.zeros((M, N), device=dev, dtype=torch.bfloat16)
    part = torch.empty((N // 128, M, 2), device=dev)
    fns = {"pf2": lambda: nat.dev_gemm_kernel(4, a, w, b, 1000 + 9102, o),
           "s3": lambda: nat.dev_gemm_kernel(4, a, w, b, 1000 + 9100, o),
           "noepi-2stage": lambda: nat.dev_gemm_kernel(4, a, w, b, 1000 + 8, o),
           "noepi-s3": lambda: nat.dev_gemm_kernel(4, a, w, b, 1000 + 9108, o),
           "st-pf2": lambda: nat.dev_gemm_ln(a, w, b, 10111, o, resid=o, st_part=part),
           "st-s3 (production)": lambda: nat.dev_gemm_ln(a, w, b, nat.EPI_RESID_FFN_BF16_ST, o, resid=o,
                                                         st_part=part)}
    res = {k: [] for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            res[k].append(timeit(f))
    flop = 2.0 * M * N * K
    print("ffn2 staging:", " | ".join(f"{k} {min(v)*1e3:7.1f} us {flop/min(v)/1e9:7.1f} TF" for k, v in res.items()),
          flush=True)


def w8b_ab(dev, g):
    """8-wave kernel with the 4-wave pipeline (gemm_bf16_w8b.hip) vs the 4-wave kernel: ffn_layer1's
    production epilogue (LN fold + GELU), the plain epilogue and no epilogue, at the forward's shapes."""
    for name, M, N, K in (("ffn1", M_TOK, 3072, 768), ("qkv", M_TOK, 2304, 768), ("ffn1-large", 65536, 4096, 1024)):
        a, w, b = operands(M, N, K, g, dev)
        o1 = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        o2 = torch.empty_like(o1)
        rs = torch.stack([torch.ones(M, device=dev), torch.zeros(M, device=dev)], 1).contiguous()
        c = torch.zeros(N, device=dev)
        nat.dev_gemm_ln(a, w, b, nat.EPI_GELU_LN, o1, ln_rs=rs, ln_c=c)
        nat.dev_gemm_w8b(a, w, b, nat.EPI_GELU_LN, o2, ln_rs=rs, ln_c=c)
        torch.cuda.synchronize()
        same = bool(torch.equal(o1, o2))
        fns = {"w4-gelu-ln": lambda: nat.dev_gemm_ln(a, w, b, nat.EPI_GELU_LN, o1, ln_rs=rs, ln_c=c),
               "w8b-gelu-ln": lambda: nat.dev_gemm_w8b(a, w, b, nat.EPI_GELU_LN, o2, ln_rs=rs, ln_c=c),
               "w4-bf16": lambda: nat.dev_gemm_kernel(4, a, w, b, 0, o1),
               "w8b-bf16": lambda: nat.dev_gemm_w8b(a, w, b, 0, o2),
               "w4-noepi": lambda: nat.dev_gemm_kernel(4, a, w, b, 1000 + 8, o1),
               "w8b-noepi": lambda: nat.dev_gemm_w8b(a, w, b, 0, o2, diag=8)}
        res = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                res[k].append(timeit(f, iters=10, warm=2))
        flop = 2.0 * M * N * K
        print(f"{name} w8b==w4 (gelu-ln): {same}: " + " | ".join(
            f"{k} {min(v)*1e3:7.1f} us {flop/min(v)/1e9:7.1f} TF" for k, v in res.items()), flush=True)
        del a, w, o1, o2


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    mode = sys.argv[1] if len(sys.argv) > 1 else ""
    if mode == "fold":
        folded(dev, g)
    elif mode == "epilds":
        variants(dev, g, 4, [0, 8, 32, 5000, 5001, 5002, 5003])
    elif mode == "grouped":
        grouped(dev, g)
    elif mode == "grouped_pmc":
        grouped_pmc(dev, g)
    elif mode == "s3":
        s3_ab(dev, g)
    elif mode == "w8b":
        w8b_ab(dev, g)
    elif mode == "skew":
        skew(dev, g)
    elif mode == "msize":
        msize(dev, g)
    elif mode == "early":
        variants(dev, g, 4, [0, 1024, 2048, 4096])
    elif mode == "nt":
        variants(dev, g, 4, [0, 256, 8])
    elif mode == "cmp":
        compare(dev, g)
        variants(dev, g, 2, [0, 1, 8, 16])
    elif mode == "ovvar":
        variants(dev, g, 2, [0, 1, 8, 16])
    elif mode == "w4var":
        variants(dev, g, 4, [0, 128, 4, 8, 136, 12])
    elif mode == "w8var":
        variants(dev, g, 8, [0, 1, 2, 8, 16])
    elif mode == "w8epi":  # 8-wave kernel with / without its epilogue (32), and without staging (33) / reads (34)
        variants(dev, g, 8, [0, 32, 33, 34])
        variants(dev, g, 4, [0, 8, 12])
    else:
        compare(dev, g)


if __name__ == "__main__":
    main()
