"""The driver's bench contract on the GPU: `python bench.py` (the configs[1] workload, a short run) prints
one JSON line with the fields the driver and the judge read -- metric / value / unit, the timing
fields, `roofline` (achieved = algorithmic FLOPs per launch / live HIP-event launch time, frac =
achieved / peak) and `traffic` quoted from the committed PMC record whenever that record was
measured on these exact sources (the fingerprint bench.py checks).  The bench runs as a child
process, as the driver runs it."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_bench_json_contract(cuda):
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline"], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["value"] > 0 and d["unit"] == "clips/s" and d["n_gpus"] == 1 and d["steps"] == 2
    assert d["dtype"] == "bf16" and d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["config"]["model"] == "videoprism_public_v1_base" and d["config"]["global_batch"] == 32
    # whole-job clips/s is B / ms_per_step
    assert abs(d["value"] - 32 / (d["ms_per_step"] / 1e3)) <= 0.01 * d["value"]
    rf = d["roofline"]
    assert rf["bound"] == "mfma" and rf["unit"] == "TFLOP/s" and rf["peak"] == 2500.0
    assert 0.0 < rf["achieved"] < rf["peak"]
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    sys.path.insert(0, os.path.join(ROOT, "videoprism-mlx_amd"))
    from videoprism import _native
    import glob
    for path in glob.glob(os.path.join(ROOT, "profiles", "traffic_r*_base.json")):
        with open(path) as f:
            rec = json.load(f)
        if rec.get("src_hash") == _native.source_fingerprint() and rf["kernel_symbol"] in rec.get("kernels", {}):
            assert rf["traffic"] is not None and rf["traffic"] > 0, rf


def test_bench_under_torchrun_world1(cuda):
    """The driver's N > 1 launch form (torch.distributed.run, rendezvous on 127.0.0.1) at one rank: the
    launcher-provided RANK / WORLD_SIZE path of bench.py (gloo group for the barrier and the max over
    ranks) prints the same contract line."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-profile"],
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["config"]["parallelism"].startswith("dp1")
