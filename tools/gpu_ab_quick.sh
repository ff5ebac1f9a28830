#!/bin/bash
# Quick library A/B on the bench without extras (lib vs lib_alt, alternating, REPS rounds, both dtypes)
# after the 2D parity tests on the default build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_fim2d.py tests/test_gpu_fullsize.py tests/test_gpu_path.py} -m gpu -q --timeout 200 --timeout-method thread > $O/abq_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/abq_tests.log; exit 1; }
tail -1 $O/abq_tests.log
for dt in ${DTYPES:-f64 f32}; do
  echo "== $dt"
  VARIANTS="lib_alt|;lib|" REPS=${REPS:-3} BENCH_ARGS="--dtype $dt --no-extra --steps 20" bash tools/gpu_ab2.sh || exit 1
done
