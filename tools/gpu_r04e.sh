# round 4: the layered solver's split-role boundary (EIK_SPLIT_WB_L, lib) against lib_v4 (off): 3D parity
# tests on lib, then an A/B on C5 (fp64 and fp32)
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fim3d.py tests/test_gpu_fm3d_early.py \
  "tests/test_gpu_fullsize.py::test_c5_full_size_properties" tests/test_gpu_arm.py > $O/r04e_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 40 $O/r04e_tests.log; exit 1; }
tail -n 2 $O/r04e_tests.log
VARIANTS="lib_v4|;lib|" REPS=3 BENCH_ARGS="--no-path --no-cpu-baseline --extras C5 --extra-steps 5 --steps 3" bash tools/gpu_ab2.sh
