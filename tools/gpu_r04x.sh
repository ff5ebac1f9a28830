# round 4: in-place pass cap for the C3 batch (default 2 for batches of > 4 maps), fp64 then fp32
export TMPDIR=/tmp
VARIANTS="lib|;lib|PASSES=4;lib|PASSES=8;lib|PASSES=16" REPS=2 BENCH_ARGS="--no-path --extras C3 --extra-steps 3 --steps 3 --warmup 1" bash tools/gpu_ab2.sh || exit 1
VARIANTS="lib|;lib|PASSES=4;lib|PASSES=8" REPS=2 BENCH_ARGS="--dtype f32 --no-path --extras C3 --extra-steps 3 --steps 3 --warmup 1" bash tools/gpu_ab2.sh || exit 1
