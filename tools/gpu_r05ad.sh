#!/bin/bash
# round 5: layered priority-band width (C5 fp64 / fp32) and C2's width 0.5 vs 1, alternating
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|PRIO=1;lib|PRIO=0.5;lib|PRIO=0.25;lib|PRIO=0.125" REPS=2 BENCH_ARGS="--no-path --steps 10 --extras C5,C5_f32 --extra-steps 5" bash tools/gpu_ab2.sh || exit 1
echo R05AD_OK
