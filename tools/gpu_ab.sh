# A/B of libeikonal builds on the bench (LIBS="lib_alt lib ...": dirs under
# planning-motion_planning_amd/, default lib_alt = baseline, lib = candidate), after the 2D solver
# GPU tests on every build.   LIBS="..." bash tools/gpu_ab.sh [bench args...]
export TMPDIR=/tmp
O=gpurun_out
LIBS=${LIBS:-"lib_alt lib"}
for v in $LIBS; do
  EIKONAL_LIB=planning-motion_planning_amd/$v/libeikonal.so timeout -k 10 300 python -u -m pytest ${AB_TESTS:-tests/test_gpu_fim2d.py} -x -q --timeout 120 --timeout-method thread > $O/ab_tests_$v.log 2>&1 || { echo "tests $v rc=$?"; tail -n 30 $O/ab_tests_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/ab_tests_$v.log)"
done
for i in 1 2; do
  for v in $LIBS; do
    EIKONAL_LIB=planning-motion_planning_amd/$v/libeikonal.so timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/ab_$v.json 2> $O/ab_$v.err || { echo "bench $v rc=$?"; tail -n 20 $O/ab_$v.err; exit 1; }
    python - "$v" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/ab_{sys.argv[1]}.json"))
r = d["roofline"]; x = d.get("extra_configs", {})
print(sys.argv[1], "C2 %.3f ms %.2f Gcells/s visits %.0f inplace %.0f path %.2f" % (d["ms_per_step"], d["value"], r["tile_visits_per_solve"], r["inplace_passes_per_solve"], d.get("ms_to_path") or 0),
      " | C3 %s" % (x.get("C3", {}).get("value")), " | costmap %s" % (x.get("costmap", {}).get("ms_per_step")), " | C4 %s | C5 %s / f32 %s" % (x.get("C4_1gpu", {}).get("value"), x.get("C5", {}).get("value"), x.get("C5_f32", {}).get("value")),
      " C5 visits %s / %s" % (x.get("C5", {}).get("tile_visits_per_solve"), x.get("C5_f32", {}).get("tile_visits_per_solve")))
PY
  done
done
