# round 4: the layered solver's first visits stage only the cost (lib: EIK_FRESH_SKIP_L=1, lib_v2: 0),
# C5 fp64 and fp32 alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="lib_v2|;lib|" REPS=3 BENCH_ARGS="--no-path --extras C5 --extra-steps 3 --steps 3 --warmup 1" bash tools/gpu_ab2.sh || exit 1
