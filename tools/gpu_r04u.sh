# round 4: EIK_EDGE_FIRST on the throughput-bound configurations (C3, C4 at one GPU) -- lib_v4 = on
export TMPDIR=/tmp
VARIANTS="lib|;lib_v4|" REPS=2 BENCH_ARGS="--no-path --extras C3,C4_1gpu --extra-steps 3 --steps 10 --warmup 2" bash tools/gpu_ab2.sh || exit 1
VARIANTS="lib|;lib_v4|" REPS=2 BENCH_ARGS="--dtype f32 --no-path --extras C3,C4_1gpu --extra-steps 3 --steps 10 --warmup 2" bash tools/gpu_ab2.sh || exit 1
