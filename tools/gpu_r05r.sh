#!/bin/bash
# round 5, final tree: the pass cap and the band width re-checked after the sweep unroll
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib|PASSES=28;lib|PASSES=56;lib|PRIO=0.7;lib|PRIO=1.4" REPS=2 BENCH_ARGS="--no-path --steps 20 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05R_OK
