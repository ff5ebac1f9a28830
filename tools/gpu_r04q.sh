export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread --durations=12 tests/test_gpu_bidir_join.py tests/test_gpu_path.py tests/test_gpu_planner.py tests/test_dropin.py > $O/r04q_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r04q_tests.log; exit 1; }
tail -n 16 $O/r04q_tests.log
