"""Handles driven from several host threads at once (include/videoprism_hip.h: one handle per thread, any
number of handles per device).  The library's launch state -- each kernel's dynamic-LDS attribute and the
CU count that sizes the persistent GEMM grids -- is kept per device and set under a lock the first time
(vp_common.h ensure_dyn_lds / device_cu_count), so two threads whose FIRST launches race must still get
the results of running one after the other, bit for bit.

The race needs a fresh process (in the test process the attributes were set long ago), so the check runs
as a child: two threads each create their own handle (bf16 and fp32, Base dims with 2 + 1 layers, and an
LvT auxiliary path) and run forwards on their own streams concurrently; then the main thread repeats the
same forwards one after the other and compares the bytes.
"""

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, threading
sys.path[:0] = [ROOT, ROOT + '/videoprism-mlx_amd']
import numpy as np, torch
from videoprism import encoders, models, params

dev = torch.cuda.current_device()
base = dict(models.CONFIGS['videoprism_v1_base'], num_spatial_layers=2, num_temporal_layers=1)
lvt = dict(models.CONFIGS['videoprism_lvt_v1_base'], vocabulary_size=100, num_spatial_layers=1,
           num_temporal_layers=1, num_auxiliary_layers=1, num_unimodal_layers=1)

def job(kind, seed):
    bf16 = kind != 'f32'
    g = torch.Generator(device='cpu').manual_seed(seed)
    if kind == 'lvt':
        var = params.synthetic_params(lvt, seed, specs=params.clip_leaf_specs(lvt))
        m = models.get_model(None, model_fn=lambda: encoders.FactorizedVideoCLIP(**lvt), fprop_dtype=torch.bfloat16)
        video = torch.rand((2, 5, 252, 252, 3), generator=g)
    else:
        var = params.synthetic_params(base, seed)
        m = models.get_model(None, model_fn=lambda: encoders.FactorizedEncoder(**base),
                             fprop_dtype=torch.bfloat16 if bf16 else None)
        video = torch.rand((2, 16, 288, 288, 3), generator=g)
    return m, var, video.to(torch.bfloat16) if bf16 else video

def run(m, var, video, eng, st):
    outs = []
    with torch.cuda.stream(st):
        x = video.to(f'cuda:{dev}', non_blocking=False)
        for _ in range(3):
            if isinstance(eng, encoders.ClipEngine):
                v = eng.encode_video(x, stream=st)[0]
            else:
                v = eng.forward(x, stream=st)[0]
            outs.append(v.clone())
    st.synchronize()
    return [o.cpu() for o in outs]

kinds = [('bf16', 1), ('f32', 2), ('lvt', 3)]
jobs = [job(k, s) for k, s in kinds]
res, errs = [None] * len(jobs), []
barrier = threading.Barrier(len(jobs))

def worker(i):
    try:
        m, var, video = jobs[i]
        eng = m.engine(var, dev)  # the handle is created in this thread
        st = torch.cuda.Stream(dev)
        barrier.wait()            # first launches of all threads at once
        res[i] = run(m, var, video, eng, st)
    except Exception as e:
        errs.append(repr(e))

ts = [threading.Thread(target=worker, args=(i,)) for i in range(len(jobs))]
[t.start() for t in ts]
[t.join() for t in ts]
assert not errs, errs
for i, (m, var, video) in enumerate(jobs):
    seq = run(m, var, video, m.engine(var, dev), torch.cuda.Stream(dev))
    for a, b in zip(res[i], seq):
        assert torch.equal(a, b), kinds[i]
    assert all(torch.equal(res[i][0], r) for r in res[i]), kinds[i]
print('threads: 3 handles on 3 threads, first launches concurrent: bitwise equal to sequential runs')
"""


@pytest.mark.timeout(300)
def test_handles_on_concurrent_threads_bitwise(cuda):
    env = dict(os.environ)
    r = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT))], env=env, capture_output=True,
                       text=True, timeout=280)
    print(r.stdout[-2000:], r.stderr[-3000:])
    assert r.returncode == 0, r.stderr[-3000:]
    assert "bitwise equal" in r.stdout
