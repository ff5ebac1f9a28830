#!/bin/bash
# round 5: layered bands by default -- the 3D / layered GPU tests, then C2 / C4 band width 0.25 / 0.5 / 1
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fim3d.py tests/test_gpu_dd_live.py tests/test_gpu_dd.py tests/test_gpu_fm3d_early.py tests/test_gpu_arm.py "tests/test_gpu_fullsize.py::test_c5_planar_matches_volume_layout" "tests/test_gpu_fullsize.py::test_c5_full_size_properties" -x -q --timeout 120 --timeout-method thread > $O/r05ae_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r05ae_tests.log; exit 1; }
tail -n 3 $O/r05ae_tests.log
VARIANTS="lib|PRIO=1;lib|PRIO=0.5;lib|PRIO=0.25" REPS=2 BENCH_ARGS="--no-path --steps 10 --extras C4_1gpu,C5 --extra-steps 6" bash tools/gpu_ab2.sh || exit 1
echo R05AE_OK
