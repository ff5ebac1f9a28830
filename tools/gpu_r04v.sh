export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_bidir_join.py tests/test_gpu_path.py tests/test_gpu_planner.py tests/test_dropin.py > $O/r04v_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 40 $O/r04v_tests.log; exit 1; }
tail -n 1 $O/r04v_tests.log
bash tools/gpu_r04n.sh
