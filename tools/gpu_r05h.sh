#!/bin/bash
# round 5: priority bands (band width = multiplier x 64 x geomean cost, front-fair dispatch) and the
# layer-planar layered solve -- probe, parity, same-box A/Bs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
EIKONAL_LIB=planning-motion_planning_amd/lib_alt/libeikonal.so timeout -k 10 120 python -u tools/prio_probe.py 0 0.5 1 2 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fim2d.py tests/test_gpu_fim3d.py tests/test_gpu_dd.py tests/test_gpu_fullsize.py -k "priority or schedule_options or planar or volume_layout or layered" -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05h_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/r05h_tests.log; exit 1; }
tail -1 $O/r05h_tests.log
VARIANTS="lib|;lib|PRIO=0.5;lib|PRIO=1;lib|PRIO=2" REPS=2 BENCH_ARGS="--no-path --steps 10 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
VARIANTS="lib|;lib|LAYER_PLANAR=1" REPS=2 BENCH_ARGS="--no-path --steps 3 --warmup 1 --extras C5 --extra-steps 3" bash tools/gpu_ab2.sh || exit 1
