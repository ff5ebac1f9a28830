#!/bin/bash
# round 5: size-scaled default band width -- the whole GPU suite, then default vs PRIO=1 on C2 / C4 / C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05ai_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r05ai_tests.log; exit 1; }
tail -n 2 $O/r05ai_tests.log
VARIANTS="lib|;lib|PRIO=1" REPS=2 BENCH_ARGS="--no-path --steps 10 --extras C4_1gpu,C5 --extra-steps 6" bash tools/gpu_ab2.sh || exit 1
echo R05AI_OK
