#!/bin/bash
# round 5: the C2 dispatch batch, small end (8 / 12 / 16 vs 32)
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib|PRIO_DISPATCH=8;lib|PRIO_DISPATCH=12;lib|PRIO_DISPATCH=16" REPS=3 BENCH_ARGS="--no-path --steps 20 --no-extra" bash tools/gpu_ab2.sh || exit 1
echo R05Z3_OK
