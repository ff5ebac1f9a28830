# round 4: A/B of the in-sweep duty steps of EIK_ASYNC_WB against the synchronous boundary (lib_alt)
export TMPDIR=/tmp
VARIANTS="lib_alt|;lib|;lib_v1|;lib_v2|;lib_v3|" REPS=2 BENCH_ARGS="--no-path --no-cpu-baseline --extras C2_other --extra-steps 10" bash tools/gpu_ab2.sh
