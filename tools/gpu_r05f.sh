#!/bin/bash
# round 5: priority bands after the end-of-solve exit fix -- quick A/B on C2 fp64 (+ C3 / C4)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fim2d.py -k "priority" -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05f_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/r05f_tests.log; exit 1; }
tail -1 $O/r05f_tests.log
VARIANTS="lib|;lib|PRIO=250;lib|PRIO=1000" REPS=2 BENCH_ARGS="--no-path --steps 10 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
