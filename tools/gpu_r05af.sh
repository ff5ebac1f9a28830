#!/bin/bash
# round 5: layered band widths on larger rasters (tools/layered_scale_probe.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u tools/layered_scale_probe.py f32 4096 8192 16384 > $O/r05af_f32.log 2>&1 || { echo "f32 rc=$?"; tail -n 20 $O/r05af_f32.log; exit 1; }
cat $O/r05af_f32.log
timeout -k 10 400 python -u tools/layered_scale_probe.py f64 4096 8192 16384 > $O/r05af_f64.log 2>&1 || { echo "f64 rc=$?"; tail -n 20 $O/r05af_f64.log; exit 1; }
cat $O/r05af_f64.log
