#!/bin/bash
# round 5, final tree (decomposition blocks: 16 x band rings): the whole GPU suite, smoke, N = 8 rehearsal
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05at_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r05at_tests.log; exit 1; }
tail -n 1 $O/r05at_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05at_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -n 20 $O/r05at_smoke.log; exit 1; }
tail -n 1 $O/r05at_smoke.log
ROUND=r05at NS="8" bash tools/gpu_c4_rehearsal.sh > $O/r05at_rehearsal.out 2>&1 || { echo "rehearsal rc=$?"; tail -n 20 $O/r05at_rehearsal.out; exit 1; }
echo R05AT_OK
