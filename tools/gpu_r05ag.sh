#!/bin/bash
# round 5: the layered solver's visit blow-up at 16384^2 -- sizes in between, another seed
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
WIDTHS=0.25 timeout -k 10 300 python -u tools/layered_scale_probe.py f32 10240 12288 14336 > $O/r05ag_a.log 2>&1 || { echo "a rc=$?"; tail -n 20 $O/r05ag_a.log; exit 1; }
cat $O/r05ag_a.log
SEED=42 WIDTHS=0.25 timeout -k 10 300 python -u tools/layered_scale_probe.py f32 8192 16384 > $O/r05ag_b.log 2>&1 || { echo "b rc=$?"; tail -n 20 $O/r05ag_b.log; exit 1; }
cat $O/r05ag_b.log
