#!/bin/bash
# round 5: priority bands on the layered solver (C5) -- parity tests, then the A/B against the FIFO
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fim3d.py -x -q --timeout 120 --timeout-method thread -k "layered" > $O/r05ac_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r05ac_tests.log; exit 1; }
tail -n 3 $O/r05ac_tests.log
VARIANTS="lib|;lib|PRIO=1;lib|PRIO=0.5;lib|PRIO=2" REPS=2 BENCH_ARGS="--no-path --steps 3 --extras C5,C5_f32 --extra-steps 5" bash tools/gpu_ab2.sh || exit 1
echo R05AC_OK
