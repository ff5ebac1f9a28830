# EIK_OPT_EXACT_BAND: its GPU parity tests (+ EXACT_TESTS), then the bench's planner step with the replay's
# per-pass trace; EXACT_AB="NAME=1 ..." adds one bench run per listed environment variant
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_bidir_exact.py ${EXACT_TESTS} > gpurun_out/exact_tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/exact_tests.log
[ $rc -le 1 ] || exit $rc
EIK_EXACT_DEBUG=1 timeout -k 10 300 python -u bench.py --no-path --extras costmap --extra-steps 4 > gpurun_out/exact_bench.json 2> gpurun_out/exact_bench.err || exit $?
i=0
for v in $EXACT_AB; do
  i=$((i+1))
  env $v EIK_EXACT_DEBUG=1 timeout -k 10 300 python -u bench.py --no-path --extras costmap --extra-steps 4 > gpurun_out/exact_bench_ab$i.json 2> gpurun_out/exact_bench_ab$i.err || exit $?
  echo "ab$i = $v"
done
echo bench ok
