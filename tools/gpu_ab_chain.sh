#!/bin/bash
# fp64 sweep-step variants (EIK_CHAIN 1 / 2 / 3 in lib_alt / lib / lib_v3): 2D parity tests on the
# default build, alternating C2 fp64 bench runs, the field error of each vs the oracle, then the
# end-effector FM3D probe (tools/arm_fm3d_probe.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fim2d.py tests/test_gpu_fullsize.py -m gpu -q --timeout 200 --timeout-method thread > $O/abc_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/abc_tests.log; exit 1; }
tail -1 $O/abc_tests.log
VARIANTS="lib_alt|;lib|;lib_v3|" REPS=${REPS:-3} BENCH_ARGS="--dtype f64 --no-extra --no-path --steps 20" bash tools/gpu_ab2.sh || exit 1
timeout -k 10 300 python tools/f64_err.py planning-motion_planning_amd/lib_v3/libeikonal.so planning-motion_planning_amd/lib/libeikonal.so 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python tools/arm_fm3d_probe.py 2>&1 | grep -v amdgpu.ids
