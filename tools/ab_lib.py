"""Same-process A/B of one kernel entry between this tree's product library and another revision's
(built by tools/ab_build.sh): both libraries are loaded side by side (ctypes, RTLD_LOCAL), fed the same
device buffers, timed in interleaved rounds, and their outputs compared bitwise.

  python tools/ab_lib.py tattn .ab/old/videoprism-mlx_amd/videoprism/libvideoprism_hip.so
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]
import torch  # noqa: E402

from videoprism import _native as nat  # noqa: E402


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


def bind(lib):
    f = lib.vp_dev_gemm_tattn
    f.restype, f.argtypes = nat._SIGNATURES["vp_dev_gemm_tattn"]
    return f


def tattn(other):
    """The fused temporal attention launches (vp_dev_gemm_tattn) at the bench shape."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    M, D, H = 131072, 768, 12
    x = (torch.rand((M, D), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand((3 * D, D), generator=g, device=dev) * 2 - 1) / D ** 0.5).to(torch.bfloat16)
    wqk, wv = w[:2 * D].contiguous(), w[2 * D:].contiguous()
    b = torch.randn(3 * D, generator=g, device=dev) * 0.1
    c = torch.randn(3 * D, generator=g, device=dev) * 0.1
    rs = torch.stack([torch.rand(M, generator=g, device=dev) + 0.5, torch.randn(M, generator=g, device=dev) * 0.1],
                     1).contiguous()
    libs = {"this": bind(nat.load()), "other": bind(ctypes.CDLL(other))}
    p = {k: torch.empty(M // 16 * H * 256, device=dev, dtype=torch.bfloat16) for k in libs}
    o = {k: torch.empty(M, D, device=dev, dtype=torch.bfloat16) for k in libs}
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())

    def qk(k):
        assert libs[k](0, ptr(x), ptr(wqk), M, D, ptr(p[k]), ptr(b), ptr(rs), ptr(c), None, H, 50.0, st()) == 0

    def vv(k):
        assert libs[k](1, ptr(x), ptr(wv), M, D, ptr(o[k]), ptr(b[2 * D:]), ptr(rs), ptr(c[2 * D:]), ptr(p[k]), H,
                       50.0, st()) == 0
    for k in libs:
        qk(k)
        vv(k)
    torch.cuda.synchronize()
    print("bitwise this == other: P", bool(torch.equal(p["this"], p["other"])), "O",
          bool(torch.equal(o["this"], o["other"])), flush=True)
    fns = {f"qk-{k}": (lambda k=k: qk(k)) for k in libs}
    fns.update({f"v-{k}": (lambda k=k: vv(k)) for k in libs})
    res = {k: [] for k in fns}
    for _ in range(4):
        for k, f in fns.items():
            res[k].append(timeit(f))
    print("tattn:", " | ".join(f"{k} {min(v)*1e3:7.1f} us" for k, v in res.items()), flush=True)


def spatial(other):
    """The spatial attention (S = 256, 12 heads, 512 frames: the bench shape) over the row-major
    q|k|v (vp_op_attention) and the row-blocked one (vp_dev_attention_spatial_blk), plus a padded
    batch (the masked kernel) and an item count that is not a multiple of the grid: bitwise this vs
    other, interleaved timing."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    H, D = 12, 768
    libs = {"this": nat.load(), "other": ctypes.CDLL(other)}
    for lib in libs.values():
        for name in ("vp_op_attention", "vp_dev_attention_spatial_blk"):
            f = getattr(lib, name)
            f.restype, f.argtypes = nat._SIGNATURES[name]
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    for nseq, blk, padded in ((512, True, False), (512, False, False), (37, True, False), (100, True, False), (16, False, True)):
        qkv = torch.randn((nseq * 256, 3 * D), generator=g, device=dev)
        qkv[:, :D] *= 0.125
        qkv = qkv.to(torch.bfloat16)
        pad = None
        if padded:
            pad = torch.zeros(nseq * 256, device=dev)
            pad[5 * 256 + 200: 6 * 256] = 1.0
        outs = {k: torch.empty((nseq * 256, D), device=dev, dtype=torch.bfloat16) for k in libs}

        def run(k):
            if blk:
                assert libs[k].vp_dev_attention_spatial_blk(ptr(qkv), ptr(outs[k]), nseq, H, 50.0, ptr(pad), st()) == 0
            else:
                assert libs[k].vp_op_attention(1, ptr(qkv), ptr(outs[k]), nseq, 256, H, 50.0, ptr(pad), st()) == 0
        for k in libs:
            run(k)
        torch.cuda.synchronize()
        same = bool(torch.equal(outs["this"], outs["other"]))
        res = {k: [] for k in libs}
        for _ in range(5):
            for k in libs:
                res[k].append(timeit(lambda k=k: run(k)))
        print(f"spatial nseq={nseq} blk={blk} padded={padded}: bitwise this == other {same}; " + " | ".join(
            f"{k} {min(v)*1e3:7.1f} us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    {"tattn": tattn, "spatial": spatial}[sys.argv[1]](sys.argv[2])
