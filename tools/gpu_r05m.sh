#!/bin/bash
# round 5: priority-band ring overflow check + FIFO fallback (lib)
# against the previous tree (lib_alt): prio tests first, then the bench A/B (C2, C3, C4).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fim2d.py tests/test_gpu_fullsize.py tests/test_gpu_dd.py tests/test_gpu_dd_live.py -x -q --timeout 200 --timeout-method thread > $O/r05m_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/r05m_tests.log; exit 1; }
tail -2 $O/r05m_tests.log
VARIANTS="lib_alt|;lib|" REPS=2 BENCH_ARGS="--no-path --steps 20 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05L_OK
