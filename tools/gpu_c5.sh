#!/bin/bash
# 3D / layered GPU tests, then the bench's C5 lines (fp64 = C5, fp32 = C5_f32).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fim3d.py tests/test_gpu_fm3d_early.py tests/test_gpu_arm.py tests/test_gpu_fullsize.py tests/test_dropin.py tests/test_gpu_planner.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/t3d2.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/t3d2.log; exit 1; }
tail -1 $O/t3d2.log
timeout -k 10 300 python bench.py --steps 3 --no-path --no-cpu-baseline --extras C5 --extra-steps 5 > $O/b5.json 2> $O/b5.err || { echo "bench rc=$?"; tail $O/b5.err; exit 1; }
python -c "
import json; d=json.load(open('$O/b5.json'))
for k,v in d['extra_configs'].items(): print(k, v)"
[ -n "$AB" ] && VARIANTS="lib_alt|;lib|" REPS=${REPS:-2} BENCH_ARGS="--steps 3 --no-path --extras C5 --extra-steps 5" bash tools/gpu_ab2.sh
true
