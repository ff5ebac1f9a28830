#!/bin/bash
# round 5: the layered solver's band dispatch batch (C5 only): 16 (default) / 32 / 48 / 64
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib|PRIO_DISPATCH=32;lib|PRIO_DISPATCH=48;lib|PRIO_DISPATCH=64" REPS=2 BENCH_ARGS="--no-path --steps 2 --extras C5 --extra-steps 8" bash tools/gpu_ab2.sh || exit 1
echo R05AK_OK
