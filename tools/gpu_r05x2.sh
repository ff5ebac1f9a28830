#!/bin/bash
# round 5: band dispatch limited by the waiting workgroups, up to 64 (lib_alt), vs 32 (lib) vs 64 (lib_v2): C2, C4 at one GPU (fp64)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
EIKONAL_LIB=planning-motion_planning_amd/lib_alt/libeikonal.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fim2d.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "prio or c4 or c2" > $O/r05x2_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/r05x2_tests.log; exit 1; }
tail -1 $O/r05x2_tests.log
VARIANTS="lib_alt|;lib|;lib_v2|" REPS=3 BENCH_ARGS="--no-path --steps 20 --extras C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05X_OK
