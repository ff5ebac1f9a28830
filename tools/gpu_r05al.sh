#!/bin/bash
# round 5: priority bands on C3 (a 128-map batch; explicit PRIO now applies to batches) and on the fp32 2D lines
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib|PRIO=0.25;lib|PRIO=1" REPS=2 BENCH_ARGS="--no-path --steps 3 --extras C3 --extra-steps 4" bash tools/gpu_ab2.sh || exit 1
VARIANTS="lib|;lib|PRIO=0.25;lib|PRIO=0.5,PRIO_DISPATCH=32" REPS=2 BENCH_ARGS="--dtype f32 --no-path --steps 10 --extras C3,C4_1gpu --extra-steps 4" bash tools/gpu_ab2.sh || exit 1
echo R05AL_OK
