# round 4: parity of the asynchronous write-back (EIK_ASYNC_WB, the default lib) on the 2D / DD /
# full-size C2 tests, then an A/B against lib_alt (EIK_ASYNC_WB=0) on the bench, alternating.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fim2d.py tests/test_gpu_dd.py \
  tests/test_gpu_fullsize.py::test_c2_full_size_fp64_vs_oracle tests/test_gpu_fullsize.py::test_c2_full_size_vs_oracle \
  "tests/test_gpu_dd_live.py::test_live_ipc_processes" tests/test_gpu_path.py tests/test_gpu_planner.py > $O/r04b_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 40 $O/r04b_tests.log; exit 1; }
tail -n 3 $O/r04b_tests.log
VARIANTS="${VARS:-lib_alt|;lib|}" REPS=${REPS:-2} BENCH_ARGS="--no-path --extras C2_other,C3,C4_1gpu --extra-steps 5" bash tools/gpu_ab2.sh
