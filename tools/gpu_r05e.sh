#!/bin/bash
# round 5: priority bands (EIK_OPT_PRIO) -- parity with the option on, then a same-box A/B of band
# widths against the FIFO (C2 fp64, C3, C4 at one GPU).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fim2d.py -k "schedule_options or priority" -m gpu -x -v --timeout 200 --timeout-method thread > $O/r05e_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/r05e_tests.log; exit 1; }
tail -2 $O/r05e_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k priority -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/r05e_tests_full.log 2>&1 || { echo "fullsize rc=$?"; tail -30 $O/r05e_tests_full.log; exit 1; }
grep -E "passed|failed|FIFO" $O/r05e_tests_full.log | tail -3
VARIANTS="lib|;lib|PRIO=250;lib|PRIO=500;lib|PRIO=1000" REPS=2 BENCH_ARGS="--no-path --steps 20 --extras C3,C4_1gpu --extra-steps 4" bash tools/gpu_ab2.sh || exit 1
