# round 4: 2D walker A/B -- EIK_PATH_SIMD0_FREE (lib_v1: the walker's SIMD partners do not build) against lib;
# the path kernel alone on the resident C2 field (bench ms_to_path fields), alternating; path parity on lib_v1 first
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
EIKONAL_LIB=planning-motion_planning_amd/lib_v1/libeikonal.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_path.py tests/test_gpu_fullsize.py::test_c2_full_size_fp64_vs_oracle > $O/r04g_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r04g_tests.log; exit 1; }
tail -n 1 $O/r04g_tests.log
for i in 1 2 3; do
  for d in lib lib_v1; do
    EIKONAL_LIB=planning-motion_planning_amd/$d/libeikonal.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 3 --warmup 1 > $O/r04g_$d.json 2> $O/r04g.err || { echo "bench $d rc=$?"; tail -n 20 $O/r04g.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/r04g_$d.json')); print('%-7s path %.3f ms  %.4f us/step  %d points  ms_to_path %.2f (torch %.2f)' % ('$d', d['path_kernel_ms'], d['path_us_per_step'], d['path_points'], d['ms_to_path'], d['ms_to_path_torch']))"
  done
done
