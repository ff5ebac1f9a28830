#!/bin/bash
# round 5: the layered solver past 4 GiB (per-tile, per-layer T buffers) -- tests, then widths by size
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest "tests/test_gpu_fullsize.py::test_c5_volume_over_4gib" "tests/test_gpu_fullsize.py::test_c5_planar_matches_volume_layout" "tests/test_gpu_fullsize.py::test_c5_full_size_properties" -x -v --timeout 200 --timeout-method thread > $O/r05ah_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r05ah_tests.log; exit 1; }
grep -E "passed|failed|over_4gib" $O/r05ah_tests.log | tail -4
WIDTHS=0,0.25,0.5,1 timeout -k 10 300 python -u tools/layered_scale_probe.py f32 16384 > $O/r05ah_f32.log 2>&1 || { echo "f32 rc=$?"; tail -n 20 $O/r05ah_f32.log; exit 1; }
cat $O/r05ah_f32.log
WIDTHS=0,0.25,0.5,1 timeout -k 10 300 python -u tools/layered_scale_probe.py f64 16384 > $O/r05ah_f64.log 2>&1 || { echo "f64 rc=$?"; tail -n 20 $O/r05ah_f64.log; exit 1; }
cat $O/r05ah_f64.log
