#!/bin/bash
# 3D solver pass: the 3D / early-exit / arm / full-size / drop-in GPU tests, then the end-effector
# probe (persistent vs list driver) and the bench's arm line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fim3d.py tests/test_gpu_fm3d_early.py tests/test_gpu_arm.py tests/test_gpu_fullsize.py tests/test_dropin.py tests/test_gpu_planner.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/t3d.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/t3d.log; exit 1; }
tail -1 $O/t3d.log
timeout -k 10 300 python tools/arm_fm3d_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python bench.py --steps 3 --no-path --no-cpu-baseline --extras arm --extra-steps 10 > $O/bench_arm.json 2> $O/bench_arm.err || { echo "bench rc=$?"; tail $O/bench_arm.err; exit 1; }
python -c "import json; print(json.load(open('$O/bench_arm.json'))['extra_configs']['arm'])"
