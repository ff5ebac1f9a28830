#!/bin/bash
# round 5: the per-solve dispatch batch (64 on maps of >= 16384 tiles, lib) vs 32 everywhere (lib_alt)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fim2d.py tests/test_gpu_fullsize.py tests/test_gpu_dd_live.py -x -q --timeout 200 --timeout-method thread > $O/r05x3_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/r05x3_tests.log; exit 1; }
tail -1 $O/r05x3_tests.log
VARIANTS="lib_alt|;lib|" REPS=3 BENCH_ARGS="--no-path --steps 20 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05X3_OK
