#!/bin/bash
# Layered-solver A/B (lib vs lib_alt) on C5, after the 3D parity tests on the default build; then the
# end-effector FM3D probe.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fim3d.py tests/test_gpu_fm3d_early.py tests/test_gpu_fullsize.py tests/test_gpu_arm.py -m gpu -q --timeout 200 --timeout-method thread > $O/ab5_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/ab5_tests.log; exit 1; }
tail -1 $O/ab5_tests.log
VARIANTS="${VARIANTS:-lib_alt|;lib|}" REPS=${REPS:-3} BENCH_ARGS="--steps 3 --no-path --extras C5 --extra-steps 5" bash tools/gpu_ab2.sh || exit 1
[ -z "$NOPROBE" ] && timeout -k 10 300 python tools/arm_fm3d_probe.py 2>&1 | grep -v amdgpu.ids
true
