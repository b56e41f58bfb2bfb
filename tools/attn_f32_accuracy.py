"""fp32 attention accuracy vs the fp64 oracle (op_attention, S = 256, 12 heads) for the library of TREE_ROOT (argv[1]):
used to A/B numerator formulations.  python tools/attn_f32_accuracy.py TREE_ROOT"""
import os, sys
root = sys.argv[1]
sys.path[:0] = [root, os.path.join(root, "videoprism-mlx_amd"), "/root/repo" if os.path.exists("/root/repo") else "."]
import numpy as np, torch
from videoprism import _native as nat
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from oracle import videoprism_oracle as orc
dev = "cuda:0"
def qkv_(num_seq, S, heads, seed, scale):
    g = torch.Generator(device="cpu").manual_seed(seed)
    D = heads * 64
    q = torch.randn(num_seq * S, D, generator=g) * scale
    k = torch.randn(num_seq * S, D, generator=g) * scale
    v = torch.randn(num_seq * S, D, generator=g)
    return torch.cat([q, k, v], dim=1)
def ref_(qkv, num_seq, S, heads, cap):
    D = heads * 64
    x = qkv.double().cpu().numpy().reshape(num_seq, S, 3, heads, 64)
    q = x[:, :, 0].transpose(0, 2, 1, 3).reshape(-1, S, 64); k = x[:, :, 1].transpose(0, 2, 1, 3).reshape(-1, S, 64)
    v = x[:, :, 2].transpose(0, 2, 1, 3).reshape(-1, S, 64)
    o = orc.capped_softmax_attention(q, k, v, cap, None)
    return o.reshape(num_seq, heads, S, 64).transpose(0, 2, 1, 3).reshape(num_seq * S, D)
for scale in (0.25, 0.5, 1.0, 2.0):
    qkv = qkv_(4, 256, 12, 7, scale).to(dev)
    out = nat.op_attention(qkv, 4, 256, 12, 50.0)
    torch.cuda.synchronize()
    err = np.abs(out.double().cpu().numpy() - ref_(qkv, 4, 256, 12, 50.0))
    print(f"{os.path.basename(root.rstrip('/'))} scale {scale}: max {err.max():.3e} mean {err.mean():.3e}", flush=True)
