# round 4: the join's 32-bit float-key sort + run fix-up -- join / path / planner / drop-in parity, phases
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bidir_join.py tests/test_gpu_path.py tests/test_gpu_planner.py tests/test_dropin.py > $O/r04p_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r04p_tests.log; exit 1; }
tail -n 1 $O/r04p_tests.log
bash tools/gpu_r04n.sh
