# round 4: first visits stage only the cost (lib: EIK_FRESH_SKIP=1, lib_v2: 0) -- GPU tests on lib,
# then C2 fp64 + C3 + C4 alternating, then fp32
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUND=r04z2 bash tools/gpu_tests.sh || exit 1
VARIANTS="lib_v2|;lib|" REPS=3 BENCH_ARGS="--no-path --extras C3,C4_1gpu --extra-steps 3 --steps 10 --warmup 2" bash tools/gpu_ab2.sh || exit 1
VARIANTS="lib_v2|;lib|" REPS=2 BENCH_ARGS="--dtype f32 --no-path --extras C3,C4_1gpu --extra-steps 3 --steps 10 --warmup 2" bash tools/gpu_ab2.sh || exit 1
