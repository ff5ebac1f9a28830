# Round-2 path walker A/B: tests of the loop forms, then tools/gpu_p2loop.sh (forms 0 1 2).
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_path.py -x -q --timeout 120 --timeout-method thread > $O/r02i_path_tests.log 2>&1; rc=$?; tail -n 3 $O/r02i_path_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_p2loop.sh
