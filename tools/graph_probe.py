"""Does the bf16 Base forward capture into a HIP graph (torch.cuda.CUDAGraph over the ctypes
launches), and what does replay save against eager launches?  Also checks that HIP events
recorded during capture (dominant-class profiling) time the replayed launches."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]
import torch  # noqa: E402

from videoprism import models, params  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    cfg = models.CONFIGS["videoprism_v1_base"]
    var = params.synthetic_params(cfg, seed=0)
    m = models.get_model("videoprism_public_v1_base", fprop_dtype=torch.bfloat16)
    eng = m.engine(var, 0)
    B = 32
    g = torch.Generator(device=dev).manual_seed(0)
    video = torch.rand((B, 16, 288, 288, 3), generator=g, device=dev).to(torch.bfloat16)
    out = torch.empty((B, 4096, 768), dtype=torch.bfloat16, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            eng.forward(video, out=out, stream=s)
    torch.cuda.synchronize()
    ref = out.clone()

    def eager(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for _ in range(k):
                eng.forward(video, out=out, stream=s)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    plain = torch.cuda.CUDAGraph()
    with torch.cuda.graph(plain, stream=s):
        eng.forward(video, out=out, stream=s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    eng.profile_only(["gemm_ffn1_gelu"])
    eng.profile_enable(64)
    with torch.cuda.graph(graph, stream=s):
        eng.forward(video, out=out, stream=s)
    torch.cuda.synchronize()

    def replay(k, gr=None):
        gr = gr or graph
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            gr.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    replay(2)
    out.zero_()
    graph.replay()
    torch.cuda.synchronize()
    print("graph output equals eager:", bool(torch.equal(out, ref)), flush=True)
    for _ in range(3):
        print(f"eager {eager(10):.3f} ms/step   graph (events) {replay(10):.3f} ms/step   "
              f"graph (no events) {replay(10, plain):.3f}", flush=True)
    replay(1)
    prof = eng.profile_read()
    print("events captured in the graph:", {k: (round(v['ms'], 3), v['launches']) for k, v in prof.items()})


if __name__ == "__main__":
    main()
