#!/bin/bash
# round 5: fp32 sweep group loop unrolled 8x (lib_alt) vs 4x (lib); fp32 bench (C2, C3, C4 at one GPU)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
EIKONAL_LIB=planning-motion_planning_amd/lib_alt/libeikonal.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_fim2d.py -x -q --timeout 200 --timeout-method thread -k "f32 or float or not f64" > $O/r05v_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/r05v_tests.log; exit 1; }
tail -1 $O/r05v_tests.log
VARIANTS="lib_alt|;lib|" REPS=3 BENCH_ARGS="--dtype f32 --no-path --steps 20 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05V_OK
