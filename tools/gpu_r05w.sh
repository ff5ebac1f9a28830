#!/bin/bash
# round 5: priority bands on a batch (C3: 128 maps, PRIO set explicitly) vs the batch's FIFO; fp64 and fp32
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib|PRIO=1;lib|PRIO=0.5" REPS=2 BENCH_ARGS="--no-path --steps 5 --extras C3 --extra-steps 3" bash tools/gpu_ab2.sh || exit 1
VARIANTS="lib|;lib|PRIO=1" REPS=2 BENCH_ARGS="--dtype f32 --no-path --steps 5 --extras C3 --extra-steps 3" bash tools/gpu_ab2.sh || exit 1
echo R05W_OK
