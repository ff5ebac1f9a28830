# round 4: in-place pass cap for the layered solver (C5; default 24), fp64
export TMPDIR=/tmp
VARIANTS="lib|;lib|PASSES=40;lib|PASSES=64;lib|PASSES=16" REPS=2 BENCH_ARGS="--no-path --extras C5 --extra-steps 3 --steps 3 --warmup 1" bash tools/gpu_ab2.sh || exit 1
