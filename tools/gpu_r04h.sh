# round 4: bounded bidirectional join (csrc/bidir.hip) -- parity vs the join's definition, the
# drop-in / planner tests that go through it, its kernels on planner step 1 (rocprofv3 stats);
# then the 2D walker A/B (EIK_PATH_SIMD0_FREE, lib_v1) of tools/gpu_r04g.sh
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  tests/test_gpu_bidir_join.py tests/test_gpu_path.py tests/test_gpu_planner.py tests/test_dropin.py \
  > $O/r04h_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 40 $O/r04h_tests.log; exit 1; }
tail -n 1 $O/r04h_tests.log
grep "k\* " $O/r04h_tests.log || true
OPTS_LIST="FRONTS_CAP=1,FRONTS_CAP=0,FRONTS_CAP=1,FRONTS_CAP=0" timeout -k 10 300 python3 tools/rover_probe.py > $O/r04h_rover_ab.log 2>&1 || { echo "rover ab rc=$?"; tail -n 20 $O/r04h_rover_ab.log; exit 1; }
grep -E "^FRONTS|bidir batch|single front" $O/r04h_rover_ab.log
OPTS_LIST="," timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r04h_prof -o rover -- python3 tools/rover_probe.py > $O/r04h_rover.log 2>&1 || { echo "rover rc=$?"; tail -n 20 $O/r04h_rover.log; exit 1; }
cat $O/r04h_rover.log | grep -v "^W\|warn" | tail -n 12
f=$(find $O/r04h_prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/r04h_rover_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04h_rover_kernel_stats.csv")))
for r in rows:
    n = r["Name"]
    if any(k in n for k in ("join", "scatter_rank", "rocprim", "bidir", "fim2d_persist", "gdm2d", "costmap")):
        print(f"{n[:90]:90s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:9.1f} us  total {float(r['TotalDurationNs'])/1e6:8.3f} ms")
PY
for i in 1 2 3; do
  for d in lib lib_v1; do
    EIKONAL_LIB=planning-motion_planning_amd/$d/libeikonal.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 3 --warmup 1 > $O/r04g_$d.json 2> $O/r04g.err || { echo "bench $d rc=$?"; tail -n 20 $O/r04g.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/r04g_$d.json')); print('%-7s C2 %.3f ms  path %.3f ms  %.4f us/step  %d points  ms_to_path %.2f (torch %.2f)' % ('$d', d['ms_per_step'], d['path_kernel_ms'], d['path_us_per_step'], d['path_points'], d['ms_to_path'], d['ms_to_path_torch']))"
  done
done
