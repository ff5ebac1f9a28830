#!/bin/bash
# Live domain decomposition on the one-GPU box: parity tests, then a 2-rank bench rehearsal
# (both ranks on cuda:0, EIK_BENCH_SHARED_GPU=1) and the single-GPU bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_gpu_dd_live.py tests/test_gpu_dd.py tests/test_gpu_fim2d.py tests/test_gpu_fim3d.py -x -q \
    > gpurun_out/live_tests.log 2>&1 || { tail -40 gpurun_out/live_tests.log; exit 1; }
tail -3 gpurun_out/live_tests.log
EIK_BENCH_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --block 2048 \
    > gpurun_out/live_bench2.log 2>&1 || { tail -40 gpurun_out/live_bench2.log; exit 1; }
tail -2 gpurun_out/live_bench2.log
EIK_BENCH_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 5 --warmup 2 --block 2048 \
    > gpurun_out/live_bench4.log 2>&1 || { tail -40 gpurun_out/live_bench4.log; exit 1; }
tail -2 gpurun_out/live_bench4.log
timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --steps 20 > gpurun_out/live_bench1.log 2>&1 \
    || { tail -40 gpurun_out/live_bench1.log; exit 1; }
tail -1 gpurun_out/live_bench1.log
EIK_BENCH_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 10 --warmup 2 \
    > gpurun_out/live_bench2_4096.log 2>&1 || { tail -40 gpurun_out/live_bench2_4096.log; exit 1; }
tail -1 gpurun_out/live_bench2_4096.log
