#!/bin/bash
# round 5: C2 fp64 (the headline raster) -- default bands vs the FIFO vs width 0.5, re-measured on the final kernels
set -o pipefail
export TMPDIR=/tmp
VARIANTS="lib|;lib|PRIO=0;lib|PRIO=0.5" REPS=3 BENCH_ARGS="--no-path --steps 20 --no-extra" bash tools/gpu_ab2.sh || exit 1
echo R05AP_OK
