# round 4: follow-through (EIK_FOLLOW) x split-role boundary (EIK_SPLIT_WB) A/B, fp64 C2 / C3 / C4
#   lib_alt: neither (the round-3 kernel); lib: both (follow max 1); v1: split only; v2: follow only; v3: both, follow max 2
export TMPDIR=/tmp
VARIANTS="lib_alt|;lib|;lib_v1|;lib_v2|;lib_v3|" REPS=2 BENCH_ARGS="--no-path --no-cpu-baseline --extras C3,C4_1gpu --extra-steps 5" bash tools/gpu_ab2.sh
