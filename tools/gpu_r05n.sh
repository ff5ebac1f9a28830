#!/bin/bash
# round 5: the sweep loop unrolled 2x (EIK_SWEEP_UNROLL=2: one back-branch per 8 steps; lib_alt) vs 1x (lib)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
EIKONAL_LIB=planning-motion_planning_amd/lib_alt/libeikonal.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "c2 or c3" > $O/r05n_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/r05n_tests.log; exit 1; }
tail -1 $O/r05n_tests.log
VARIANTS="lib_alt|;lib|" REPS=3 BENCH_ARGS="--no-path --steps 20 --extras C2_f32,C3,C4_1gpu,C5 --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05N_OK
