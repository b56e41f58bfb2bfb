"""Throughput of the fp32 forward (fprop_dtype=None: the reference's default precision, models.py:268-303):
Base (or Large) at B clips x 16 x 288 x 288 on one GPU, with the per-class kernel breakdown from the
library's HIP-event profiler.  Measurement only (the bench's headline is bf16)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "videoprism-mlx_amd")]
import torch  # noqa: E402

from videoprism import models, params  # noqa: E402


def main(name="videoprism_public_v1_base", B=4, steps=3):
    cfg_key = {"videoprism_public_v1_base": "videoprism_v1_base",
               "videoprism_public_v1_large": "videoprism_v1_large"}[name]
    cfg = dict(models.CONFIGS[cfg_key])
    model = models.get_model(name)  # fp32
    var = params.synthetic_params(cfg, seed=0)
    eng = model.engine(var, 0)
    video = torch.rand((B, 16, 288, 288, 3), device="cuda:0")
    out = torch.empty((B, 16 * 256, cfg["model_dim"]), device="cuda:0")
    eng.forward(video, out=out)
    torch.cuda.synchronize()
    eng.profile_enable(512)
    eng.forward(video, out=out)
    torch.cuda.synchronize()
    br = eng.profile_read()
    eng.profile_enable(0)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.forward(video, out=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    gpc = 973.29 if "base" in name else None
    res = {"model": name, "dtype": "f32", "B": B, "ms_per_step": round(dt * 1e3, 2), "clips_per_s": round(B / dt, 2),
           "tflops_whole_forward": round(B * gpc / dt / 1e3, 1) if gpc else None,
           "kernels": {k: {"ms": round(v["ms"], 3), "launches": v["launches"],
                           "tflops": round(v["flops"] / v["ms"] / 1e9, 1) if v["flops"] else None}
                       for k, v in sorted(br.items(), key=lambda kv: -kv[1]["ms"])}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*(sys.argv[1:2] or []), *([int(a) for a in sys.argv[2:4]]))
