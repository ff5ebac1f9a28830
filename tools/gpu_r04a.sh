# round 4, first GPU pass: the new parity tests (fp64 C3 / C4, the C4 4x2 split at 4096^2, the
# ADVICE regressions), then the bench line with the new fields.
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dd.py::test_solve_then_merge_then_iterate tests/test_gpu_dd.py::test_nan_cost_blocks_fp64_device \
  tests/test_gpu_fim3d.py::test_layered_nan_cost_blocks tests/test_gpu_fullsize.py \
  tests/test_gpu_dd_live.py::test_c4_split_4x2_assembled_field > $O/r04a_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 40 $O/r04a_tests.log; exit 1; }
timeout -k 10 600 python bench.py > $O/r04a_bench.json 2> $O/r04a_bench.err || { echo "bench rc=$?"; tail -n 20 $O/r04a_bench.err; exit 1; }
echo ALLOK
