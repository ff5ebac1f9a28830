#!/bin/bash
# round 5: priority bands in fp32 again, with the per-solve dispatch batch (PRIO=1) vs the fp32 FIFO default
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib|PRIO=1" REPS=2 BENCH_ARGS="--dtype f32 --no-path --steps 20 --extras C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05Y2_OK
