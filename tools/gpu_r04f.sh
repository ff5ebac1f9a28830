# round 4: EIK_LAZY_CLAIM (lib_v1) -- 2D parity tests on it, then an A/B against lib (the round-3 schedule)
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
EIKONAL_LIB=planning-motion_planning_amd/lib_v1/libeikonal.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fim2d.py tests/test_gpu_dd.py "tests/test_gpu_dd_live.py::test_live_ipc_processes" \
  tests/test_gpu_fullsize.py::test_c2_full_size_fp64_vs_oracle tests/test_gpu_path.py tests/test_gpu_planner.py > $O/r04f_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 40 $O/r04f_tests.log; exit 1; }
tail -n 2 $O/r04f_tests.log
VARIANTS="lib|;lib_v1|" REPS=3 BENCH_ARGS="--no-path --no-cpu-baseline --extras C2_other,C3,C4_1gpu --extra-steps 5" bash tools/gpu_ab2.sh
