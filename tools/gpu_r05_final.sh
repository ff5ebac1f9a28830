#!/bin/bash
# round 5, final tree: the round's evidence pass (tools/gpu_round.sh: GPU tests, smoke, bench line,
# kernel stats, PMC traffic of C2 and C5) and the SQ counters of the fp64 headline kernel with the
# priority bands.   ROUND=r05b bash tools/gpu_r05_final.sh
set -o pipefail
export TMPDIR=/tmp
R=${ROUND:-r05b}
O=gpurun_out
mkdir -p $O
ROUND=$R DTYPE=f64 bash tools/gpu_round.sh || exit 1
O=/tmp bash tools/gpu_pmc_sq.sh || exit 1
python tools/sq_summary.py /tmp/pmcsq1.csv /tmp/pmcsq2.csv --kernel "fim2d_persist_kernel<double" --label "C2 fp64 headline, priority bands ($R)" > $O/${R}_sq_counters.json || exit 1
echo FINAL_OK
