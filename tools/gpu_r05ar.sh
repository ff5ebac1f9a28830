#!/bin/bash
# round 5, final tree (DD blocks at band width >= 1): the whole GPU suite and the smoke test
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05ar_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r05ar_tests.log; exit 1; }
tail -n 1 $O/r05ar_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05ar_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -n 20 $O/r05ar_smoke.log; exit 1; }
tail -n 1 $O/r05ar_smoke.log
