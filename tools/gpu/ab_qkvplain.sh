#!/bin/bash
# A/B: q|k|v projection store mode (nontemporal / plain) x spatial attention order (forward / reverse)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r03q_base_$i.log 2>&1 || exit 1
  VP_QKV_PLAIN=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r03q_plain_$i.log 2>&1 || exit 1
  VP_QKV_PLAIN=1 VP_ATTN_REV=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r03q_plainrev_$i.log 2>&1 || exit 1
  VP_ATTN_REV=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r03q_rev_$i.log 2>&1 || exit 1
done
