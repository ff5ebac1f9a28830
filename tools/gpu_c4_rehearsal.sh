#!/bin/bash
# C4 as BASELINE configs[3] names it (one 16384^2 raster, seed 7, goal at the centre, split 2x1 /
# 2x2 / 4x2), rehearsed on the one-GPU box: every rank on cuda:0 (EIK_BENCH_SHARED_GPU=1, gloo
# world group, co-resident grids split between the ranks).  Checks that bench.py's N > 1 path
# emits the strong-scaling line (H = W = 16384, split, dd_mode, halo transport, C3_sharded); the
# timings are NOT a scaling measurement (the ranks share one GPU).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=${ROUND:-r03}
for n in ${NS:-2 4 8}; do
  EIK_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus $n --steps ${STEPS:-3} --warmup 1 \
      ${BENCH_ARGS:-} > gpurun_out/${R}_c4_rehearsal_n$n.log 2>&1 || { echo "n=$n rc=$?"; tail -40 gpurun_out/${R}_c4_rehearsal_n$n.log; exit 1; }
  grep '^{' gpurun_out/${R}_c4_rehearsal_n$n.log | tail -1
done
