#!/bin/bash
# round 5: the band dispatch batch sized by the waiting workgroups (lib_w: EIK_DISP_WAITERS=1) vs lib
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib_w|" REPS=2 BENCH_ARGS="--no-path --steps 10 --extras C4_1gpu,C5 --extra-steps 4" bash tools/gpu_ab2.sh || exit 1
VARIANTS="lib|;lib_w|;lib_w|PRIO=0.25;lib_w|PRIO=0.5" REPS=2 BENCH_ARGS="--dtype f32 --no-path --steps 10 --extras C4_1gpu --extra-steps 4" bash tools/gpu_ab2.sh || exit 1
echo R05AM_OK
