#!/bin/bash
# round 5: fp64 2D band widths at 1024^2 / 2048^2 / 8192^2 (default -1 = default_prio, 0 = FIFO)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u tools/prio_size_probe_2d.py 1024 2048 8192 > $O/r05an.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r05an.log; exit 1; }
cat $O/r05an.log
timeout -k 10 300 python -u tools/prio_size_probe_2d.py 1024 2048 8192 > $O/r05an2.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r05an2.log; exit 1; }
cat $O/r05an2.log
