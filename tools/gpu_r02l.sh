# Round-2 3D walker check: 3D/arm/planner parity tests, the C5 full-size test, walker timing.
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fim3d.py tests/test_gpu_arm.py tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread > $O/r02l_p3_tests.log 2>&1; rc=$?; tail -n 3 $O/r02l_p3_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/r02l_p3_tests.log | head -20; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "C5 or c5 or layered or 3d" > $O/r02l_full_tests.log 2>&1; rc=$?; tail -n 3 $O/r02l_full_tests.log; [ $rc -eq 0 ] || exit 1
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DP3_NOPROBE tools/path3_prof.hip -o /tmp/p3n && timeout -k 10 60 /tmp/p3n
timeout -k 10 120 python tools/path3_bench.py
