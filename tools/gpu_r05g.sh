#!/bin/bash
# priority bands (oldest-waiter dispatch): probe with queue counters, then parity, then a quick A/B
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out
mkdir -p $O
EIKONAL_LIB=planning-motion_planning_amd/lib_alt/libeikonal.so timeout -k 10 120 python -u tools/prio_probe.py 0 0.25 0.5 1 2 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fim2d.py -k "priority or schedule_options" -m gpu -x -q --timeout 100 --timeout-method thread > $O/r05g_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/r05g_tests.log; exit 1; }
tail -1 $O/r05g_tests.log
VARIANTS="lib|;lib|PRIO=0.25;lib|PRIO=0.5;lib|PRIO=1;lib|PRIO=2" REPS=2 BENCH_ARGS="--no-path --steps 10 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
