#!/bin/bash
# round 5, final tree: C3's in-place pass cap (a batch's default 2) 1 / 3 / 4
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib|PASSES=1;lib|PASSES=3;lib|PASSES=4" REPS=2 BENCH_ARGS="--no-path --steps 3 --extras C3 --extra-steps 3" bash tools/gpu_ab2.sh || exit 1
VARIANTS="lib|;lib|PASSES=3" REPS=2 BENCH_ARGS="--dtype f32 --no-path --steps 3 --extras C3 --extra-steps 3" bash tools/gpu_ab2.sh || exit 1
echo R05AB_OK
