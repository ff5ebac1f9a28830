#!/bin/bash
# round 5: where the 4x2 live decomposition's extra work comes from -- the C4 rehearsal (16384^2
# fp64, 8 ranks sharing the one GPU) with every rank's visits / passes in the line (dd_per_rank),
# the default (priority bands in fp64) against the FIFO (PRIO=0).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "" "PRIO=0"; do
  tag=${v:-default}; tag=${tag//[^A-Za-z0-9]/_}
  EIK_OPTIONS="$v" EIK_BENCH_SHARED_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port 29788 bench.py --gpus 8 --steps 2 --warmup 1 --no-extra \
      > gpurun_out/r05d_c4_n8_$tag.log 2>&1 || { echo "$tag rc=$?"; tail -30 gpurun_out/r05d_c4_n8_$tag.log; exit 1; }
  grep '^{' gpurun_out/r05d_c4_n8_$tag.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']
print('$tag', d['ms_per_step'], 'ms', c.get('dd_field_ok'), c.get('dd_rounds_per_solve'), json.dumps(c.get('dd_per_rank')), c.get('single_domain_tile_visits'), c.get('single_domain_inplace_passes'))"
done
echo R05D_OK
