#!/bin/bash
# round 5, final tree: a waiter's poll sleep 1 (lib_alt) vs 4 (lib), and the band width 0.7 / 1.4 (C2, C4 fp64)
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib_alt|;lib|PRIO=0.7;lib|PRIO=1.4" REPS=2 BENCH_ARGS="--no-path --steps 20 --extras C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05AA_OK
