#!/bin/bash
# round 5: long clips, patch sizes, misaligned frames, production-shape oracle gate, T<=32 bitwise A/B
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread \
  tests/test_gpu_long_clips.py tests/test_gpu_geometry.py \
  "tests/test_gpu_kernels.py::test_patch_embed_fused_from_frames" \
  "tests/test_gpu_kernels.py::test_patch_embed_fused_rejects_odd_patch" \
  "tests/test_gpu_fullsize.py::test_production_shape_layers_vs_wbf16_oracle" \
  "tests/test_gpu_fullsize.py::test_fullsize_batch_properties_bf16" -s > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab_forward_hash.py > $O/hash_this.json 2> $O/hash_this.err && \
timeout -k 10 300 python tools/ab_forward_hash.py .ab/r04 > $O/hash_r04.json 2> $O/hash_r04.err
echo "hash rc=$?"
