#!/bin/bash
# round 5: EIK_EDGE_FIRST=1 with the edge-column copies (only T's rows 0 / 63 and the W / E copies
# drained before the activations; interior rows incl. T's edge columns drained during the next
# sweep) (lib_alt) vs the default write-back (lib).  C2 is throughput-bound in its middle phase
# (the trace: 80 % of pushes find no waiting workgroup), so a pass's drain costs solve time.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
EIKONAL_LIB=planning-motion_planning_amd/lib_alt/libeikonal.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_fim2d.py tests/test_gpu_dd.py -x -q --timeout 200 --timeout-method thread > $O/r05t_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/r05t_tests.log; exit 1; }
tail -1 $O/r05t_tests.log
VARIANTS="lib_alt|;lib|" REPS=3 BENCH_ARGS="--no-path --steps 20 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05T_OK
