#!/bin/bash
# round 5: priority bands on layered decomposition blocks -- the layered DD tests, then FIFO vs bands
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dd.py tests/test_gpu_dd_live.py -x -q --timeout 200 --timeout-method thread > $O/r05as_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r05as_tests.log; exit 1; }
tail -n 1 $O/r05as_tests.log
timeout -k 10 300 python -u tools/dd_layered_probe.py 2048 2 2 > $O/r05as_probe.log 2>&1 || { echo "probe rc=$?"; tail -n 20 $O/r05as_probe.log; exit 1; }
cat $O/r05as_probe.log
