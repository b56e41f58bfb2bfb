#!/bin/bash
# Whole-forward A/B on one box: this tree's bench.py and another revision's (built by tools/ab_build.sh
# into .ab/NAME), alternating, ROUNDS rounds each; every run its own time limit, stop at the first failure.
#   bash tools/gpu/ab_bench.sh NAME [ROUNDS] [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
NAME=$1
ROUNDS=${2:-3}
shift 2
for r in $(seq 1 "$ROUNDS"); do
  for side in this "$NAME"; do
    dir=.
    [ "$side" = this ] || dir=".ab/$NAME"
    timeout -k 10 300 python -u "$dir/bench.py" --no-cpu-baseline "$@" > "gpurun_out/ab_${side}_$r.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "ab_bench: $side round $r rc=$rc"; tail -5 "gpurun_out/ab_${side}_$r.log"; exit $rc; }
    python - "$side" "gpurun_out/ab_${side}_$r.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(f"{sys.argv[1]:8s} {d['value']:8.1f} clips/s  {d['ms_per_step']:7.3f} ms/step  " +
      " ".join(f"{k} {v:.3f}" for k, v in d["kernel_ms_per_step"].items()), flush=True)
PY
  done
done
