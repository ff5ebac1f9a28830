#!/bin/bash
# round 5: EIK_EARLY_AND (activation consumption inside the sweep, halo reload beside the write-back):
# parity on lib_alt (step 96), then a same-box A/B against the default build and lib_v2 (step 64).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
EIKONAL_LIB=planning-motion_planning_amd/lib_alt/libeikonal.so timeout -k 10 500 python -u -m pytest tests/test_gpu_fim2d.py tests/test_gpu_fullsize.py tests/test_gpu_dd.py tests/test_gpu_dd_live.py tests/test_gpu_bidir_join.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05b_tests_alt.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/r05b_tests_alt.log; exit 1; }
tail -2 $O/r05b_tests_alt.log
VARIANTS="lib|;lib_alt|;lib_v2|" REPS=3 BENCH_ARGS="--no-path --steps 20 --extras C3,C4_1gpu,C2_other --extra-steps 4" bash tools/gpu_ab2.sh || exit 1
