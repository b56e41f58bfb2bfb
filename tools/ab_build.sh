#!/bin/bash
# Builds the product library of another revision for same-box A/B runs (tools/ab_lib.py, and
# tools/gpu/ab_bench.sh, which runs that revision's bench.py alternately with this tree's):
#   bash tools/ab_build.sh REV NAME   ->   .ab/NAME/videoprism-mlx_amd/videoprism/libvideoprism_hip.so
# (.ab/ is git-ignored; its libraries travel to the GPU box with the tree, its objects do not)
set -e
cd "$(dirname "$0")/.."
REV=$1
NAME=$2
rm -rf ".ab/$NAME"
mkdir -p ".ab/$NAME"
git archive "$REV" videoprism-mlx_amd include tools oracle bench.py __graft_entry__.py | tar -x -C ".ab/$NAME"
make -C ".ab/$NAME/videoprism-mlx_amd" -j8 > ".ab/$NAME/build.log" 2>&1 || { tail -5 ".ab/$NAME/build.log"; exit 1; }
echo ".ab/$NAME/videoprism-mlx_amd/videoprism/libvideoprism_hip.so"
