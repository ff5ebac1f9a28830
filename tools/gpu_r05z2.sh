#!/bin/bash
# round 5: the dispatch batch swept with EIK_OPT_PRIO_DISPATCH: C2 (16 / 24 / 32 / 48) and C4 at one GPU (48 / 64)
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib|PRIO_DISPATCH=16;lib|PRIO_DISPATCH=24;lib|PRIO_DISPATCH=48" REPS=2 BENCH_ARGS="--no-path --steps 20 --no-extra" bash tools/gpu_ab2.sh || exit 1
VARIANTS="lib|;lib|PRIO_DISPATCH=48" REPS=2 BENCH_ARGS="--no-path --steps 5 --extras C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05Z2_OK
