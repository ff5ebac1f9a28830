#!/bin/bash
# round 5: the 3D walker's run loop with one exit branch per step (EIK_P3ONE=1, lib) vs the
# multi-exit loop (lib_alt): 3D path tests, the tool's timing, the bench's C5 path
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_path.py tests/test_gpu_fim3d.py tests/test_gpu_fullsize.py tests/test_gpu_planner.py -x -q --timeout 200 --timeout-method thread > $O/r05q_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/r05q_tests.log; exit 1; }
tail -1 $O/r05q_tests.log
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DP3_NOPROBE tools/path3_prof.hip -o /tmp/p3new || exit 1
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DP3_NOPROBE -DEIK_P3ONE=0 tools/path3_prof.hip -o /tmp/p3old || exit 1
for r in 1 2; do
  echo "one-exit:  $(timeout -k 10 60 /tmp/p3new | tr '\n' ' ')"
  echo "multi-exit: $(timeout -k 10 60 /tmp/p3old | tr '\n' ' ')"
done
for L in lib lib_alt lib lib_alt; do
  EIKONAL_LIB=planning-motion_planning_amd/$L/libeikonal.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-path --no-timing --extras C5,arm --extra-steps 3 > /tmp/b_$L.json 2> /tmp/b_$L.err || { echo "bench rc=$?"; tail /tmp/b_$L.err; exit 1; }
  python -c "import json;d=json.load(open('/tmp/b_$L.json'))['extra_configs'];print('$L', 'C5 path_ms_device', d['C5']['path_ms_device'], 'points', d['C5']['path_points'], 'arm', d['arm'].get('ms_volume_fm3d_path'))"
done
echo R05Q_OK
