#!/bin/bash
# round 5: queue entries with state hints + the FIFO words loaded beside the state atomics (lib)
# against the previous tree (lib_alt): prio tests first, then the bench A/B (C2, C3, C4).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fim2d.py tests/test_gpu_fullsize.py tests/test_gpu_dd.py tests/test_gpu_dd_live.py -x -q --timeout 200 --timeout-method thread > $O/r05l_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/r05l_tests.log; exit 1; }
tail -2 $O/r05l_tests.log
VARIANTS="lib_alt|;lib|" REPS=3 BENCH_ARGS="--no-path --steps 20 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
echo R05L_OK
