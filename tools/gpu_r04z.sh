# round 4: fp64 layered tile height (C5): lib 40 rows (1 workgroup / CU), lib_v2 12 rows and lib_v3 8 rows
# (2 workgroups / CU), alternating; fp64 then fp32 (fp32 unaffected: 64 rows)
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="lib|;lib_v2|;lib_v3|" REPS=2 BENCH_ARGS="--no-path --extras C5 --extra-steps 3 --steps 3 --warmup 1" bash tools/gpu_ab2.sh || exit 1
