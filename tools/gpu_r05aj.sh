#!/bin/bash
# round 5: layered solver with bands -- dispatch batch and in-place pass cap re-checked (C5 only)
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib|PRIO_DISPATCH=32;lib|PRIO_DISPATCH=8;lib|PASSES=12;lib|PASSES=48" REPS=2 BENCH_ARGS="--no-path --steps 2 --extras C5 --extra-steps 6" bash tools/gpu_ab2.sh || exit 1
echo R05AJ_OK
