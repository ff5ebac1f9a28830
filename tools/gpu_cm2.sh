#!/bin/bash
# cost builder + planner tests, then the rover path probe and the bench's costmap line
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_costmap.py tests/test_gpu_planner.py -m gpu -q -x --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
OPTS_LIST="" timeout -k 10 300 python tools/rover_probe.py 2>&1 | grep default || exit 1
timeout -k 10 300 python bench.py --steps 2 --no-path --no-cpu-baseline --extras costmap --extra-steps 5 2>/dev/null > gpurun_out/bcm.json || exit 1
python -c "import json; d=json.load(open('gpurun_out/bcm.json')); print(d['extra_configs']['costmap'])"
