export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_costmap.py tests/test_costmap_oracle.py -x -q > gpurun_out/t_cm.log 2>&1; rc=$?; tail -n 40 gpurun_out/t_cm.log; exit $rc
