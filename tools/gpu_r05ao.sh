#!/bin/bash
# round 5: where the bands start to pay -- fp64 2D at 2560^2 / 3072^2 / 3584^2, layered at 1024^2 / 2048^2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
WIDTHS=0,0.25 timeout -k 10 300 python -u tools/prio_size_probe_2d.py 2560 3072 3584 4096 > $O/r05ao_2d.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r05ao_2d.log; exit 1; }
cat $O/r05ao_2d.log
WIDTHS=0,0.25 timeout -k 10 300 python -u tools/layered_scale_probe.py f32 1024 2048 3072 > $O/r05ao_l32.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r05ao_l32.log; exit 1; }
cat $O/r05ao_l32.log
WIDTHS=0,0.25 timeout -k 10 300 python -u tools/layered_scale_probe.py f64 1024 2048 3072 > $O/r05ao_l64.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r05ao_l64.log; exit 1; }
cat $O/r05ao_l64.log
