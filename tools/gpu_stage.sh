#!/bin/bash
# host-entry tests after the pinned-staging change, then the drop-in / rover timings
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_stage.log 2>&1 || { tail -30 gpurun_out/t_stage.log; exit 1; }
tail -1 gpurun_out/t_stage.log
OPTS_LIST="," timeout -k 10 300 python tools/rover_probe.py 2>&1 | grep -E "default|bidir" && FRESH=1 OPTS_LIST="," timeout -k 10 300 python tools/rover_probe.py 2>&1 | grep -E "default|bidir"
