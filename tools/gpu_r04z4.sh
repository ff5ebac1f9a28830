# round 4: C2 fp64 one-map pass cap (default 40) re-checked with the first-visit staging
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="lib|;lib|PASSES=32;lib|PASSES=56" REPS=3 BENCH_ARGS="--no-path --no-extra --steps 10 --warmup 2" bash tools/gpu_ab2.sh || exit 1
