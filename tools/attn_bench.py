"""Spatial attention microbenchmark at the bench shape (B=32 clips x 16 frames = 512 sequences
of 256 tokens, 12 heads): the production kernel against a q|k|v-sized copy (the memory stream's
ceiling); interleaved rounds in one process.  `long`: the LvT auxiliary attention and its diag-library
A/B builds.  (The ablation builds and the half-frame kernel that priced its parts are recorded in
profiles/HISTORY.md; their sources are in git history.)"""
import os
import sys

if sys.argv[1:2] == ["long"]:
    os.environ.setdefault("VP_DIAG_LIB", "1")  # the A/B builds live in the diag library

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


def main():
    dev = torch.device("cuda:0")
    nseq, heads, S = 512, 12, 256
    g = torch.Generator(device=dev).manual_seed(0)
    D = heads * 64
    qkv = torch.randn((nseq * S, 3 * D), generator=g, device=dev)
    qkv[:, :D] *= 0.125
    qkv = qkv.to(torch.bfloat16)
    o = torch.empty((nseq * S, D), device=dev, dtype=torch.bfloat16)
    fns = {"prod": lambda: nat.op_attention(qkv, nseq, S, heads, 50.0, out=o)}
    # streaming reference: read the q|k|v buffer and write a same-size copy (2 x 604 MB)
    cp = torch.empty_like(qkv)
    fns["copy"] = lambda: cp.copy_(qkv)
    res = {k: [] for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            res[k].append(timeit(f))
    flop = 4.0 * nseq * S * S * D
    nbytes = qkv.numel() * 2
    print(f"copy of q|k|v: {2 * nbytes / min(res['copy']) / 1e6:.0f} GB/s; attention bytes "
          f"{(nbytes + o.numel() * 2) / 1e6:.0f} MB", flush=True)
    print("spatial attention:", " ".join(f"{k}: {min(v)*1e3:6.1f} us ({flop/min(v)/1e9:5.0f} TF)"
                                        for k, v in res.items()), flush=True)


def long_variants():
    """The auxiliary (4096-token) attention at the LvT-Large bench shape (32 clips x 16 heads, S = 4096):
    the product kernel (var 0) against its diag-library A/B builds (attention_long_kernel.h VAR bits:
    8: without the linear tier for |logit| <= 0.10 cap = round 4's kernel; 16: row sum on the MFMA;
    32: row sum by v_dot2_f32_bf16; 64: unpaired scalar numerator and row sum; 80, 96 combined), at three
    logit scales (std 0.5 / 2 / 6: linear, quadratic / cubic and mixed tiers), interleaved rounds.
    VP_DIAG_LIB=1 python tools/attn_bench.py long   (VP_ATTN_VARIANTS=0,8 picks the builds)"""
    dev = torch.device("cuda:0")
    nseq, heads, S = 32, 16, 4096
    D = heads * 64
    st = lambda: torch.cuda.current_stream().cuda_stream
    variants = tuple(int(v) for v in os.environ.get("VP_ATTN_VARIANTS", "0,8,16,32,64,80,96").split(","))
    for qscale in (0.0625, 0.25, 0.75):
        g = torch.Generator(device=dev).manual_seed(0)
        qkv = torch.randn((nseq * S, 3 * D), generator=g, device=dev)
        qkv[:, :D] *= qscale
        qkv = qkv.to(torch.bfloat16)
        outs, fns = {}, {}
        for var in variants:
            outs[var] = torch.empty((nseq * S, D), device=dev, dtype=torch.bfloat16)
            fns[f"var{var}"] = (lambda var=var: nat.call("vp_dev_attention_long_var", var, qkv.data_ptr(),
                                                         outs[var].data_ptr(), nseq, S, heads, 50.0, st()))
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        ref = outs[0].float()
        print(f"logit std {qscale * 8:.1f}: " + " ".join(
            f"var{v} vs var0 max {(outs[v].float() - ref).abs().max().item():.2e} (bitwise {bool(torch.equal(outs[v], outs[0]))})"
            for v in variants[1:]), flush=True)
        res = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                res[k].append(timeit(f, iters=5, warm=1))
        flop = 4.0 * nseq * S * S * D
        print("aux attention:", " ".join(f"{k}: {min(v):7.3f} ms ({flop/min(v)/1e9:5.0f} TF)" for k, v in res.items()),
              flush=True)
        del qkv, outs


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "long":
        long_variants()
    else:
        main()
