# round 4: planner step 1 with the device min(Z) in the host assembly: planner / drop-in tests, phases
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planner.py tests/test_dropin.py tests/test_gpu_costmap.py > $O/r04o_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r04o_tests.log; exit 1; }
tail -n 1 $O/r04o_tests.log
bash tools/gpu_r04n.sh
