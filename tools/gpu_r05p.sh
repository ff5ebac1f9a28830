#!/bin/bash
# round 5: the layered sweep's group loop unrolled 1x (lib), 2x (lib_alt), 4x (lib_v2); fim2d at 4x in all
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for L in lib_alt lib_v2; do
EIKONAL_LIB=planning-motion_planning_amd/$L/libeikonal.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fim3d.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "layered or c5" > $O/r05p_tests_$L.log 2>&1 || { echo "tests $L rc=$?"; tail -20 $O/r05p_tests_$L.log; exit 1; }
tail -1 $O/r05p_tests_$L.log
done
VARIANTS="lib|;lib_alt|;lib_v2|" REPS=2 BENCH_ARGS="--no-path --steps 10 --extras C5 --extra-steps 3" bash tools/gpu_ab2.sh || exit 1
echo R05P_OK
