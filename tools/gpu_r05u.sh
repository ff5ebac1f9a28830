#!/bin/bash
# round 5: C2 / C3 / C4 fp64 against the persistent grid (EIK_OPT_GRID: 256 = 1 workgroup per CU,
# 384, 512 = the default 2 per CU) -- how much residency buys in the throughput-bound phase
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|GRID=256;lib|GRID=384;lib|;lib|GRID=448" REPS=2 BENCH_ARGS="--no-path --steps 20 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05U_OK
