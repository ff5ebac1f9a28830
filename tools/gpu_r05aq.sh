#!/bin/bash
# round 5: FIFO default below the size threshold -- the whole GPU suite, then small rasters default vs FIFO
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05aq_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r05aq_tests.log; exit 1; }
tail -n 2 $O/r05aq_tests.log
WIDTHS=-1,0 timeout -k 10 300 python -u tools/prio_size_probe_2d.py 1024 2048 4096 > $O/r05aq_2d.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r05aq_2d.log; exit 1; }
cat $O/r05aq_2d.log
WIDTHS=-1,0 timeout -k 10 300 python -u tools/layered_scale_probe.py f64 2048 4096 > $O/r05aq_l64.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r05aq_l64.log; exit 1; }
cat $O/r05aq_l64.log
