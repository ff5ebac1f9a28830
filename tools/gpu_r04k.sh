# round 4: EIK_ECOL A/B in fp32 (C2 fp32, C4 at one GPU fp32: the 4-wave kernel, which spills 13 VGPRs with ECOL)
export TMPDIR=/tmp
VARIANTS="lib|;lib_v3|" REPS=3 BENCH_ARGS="--dtype f32 --no-path --extras C4_1gpu --extra-steps 3 --steps 10 --warmup 2" bash tools/gpu_ab2.sh || exit 1
