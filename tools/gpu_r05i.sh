#!/bin/bash
# priority bands without the front reserve: probe + A/B (C2, C3, C4) of the band-width multiplier
set -o pipefail
export TMPDIR=/tmp
EIKONAL_LIB=planning-motion_planning_amd/lib_alt/libeikonal.so timeout -k 10 120 python -u tools/prio_probe.py 0 0.5 1 2 || exit 1
N=16384 EIKONAL_LIB=planning-motion_planning_amd/lib_alt/libeikonal.so timeout -k 10 200 python -u tools/prio_probe.py 0 0.5 1 2 || exit 1
VARIANTS="lib|;lib|PRIO=0.5;lib|PRIO=1;lib|PRIO=2" REPS=2 BENCH_ARGS="--no-path --steps 10 --extras C3,C4_1gpu --extra-steps 2" bash tools/gpu_ab2.sh || exit 1
