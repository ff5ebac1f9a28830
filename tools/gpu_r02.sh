# Round-2 iteration: GPU tests, event traces (DEM + uniform), bench lines.  TAG names the outputs;
# AB="opt1;opt2" runs the bench (and trace) once per EIK_OPTIONS value ("-" = defaults), twice.
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-r02}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -n 40 $O/${TAG}_gpu_tests.log; exit 1; }
tail -n 2 $O/${TAG}_gpu_tests.log
fi
IFS=';' read -ra VARS <<< "${AB:--}"
summ() {
python - "$1" "$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]; x = d.get("extra_configs", {})
print(sys.argv[2], "C2 %.3f ms %.2f Gcells/s frac %.4f visits %.0f inplace %.0f path %.2f" % (d["ms_per_step"], d["value"], r["frac"], r["tile_visits_per_solve"], r["inplace_passes_per_solve"], d.get("ms_to_path") or 0),
      "| C3 %s | C4 %s | C5 %s" % (x.get("C3", {}).get("value"), x.get("C4_1gpu", {}).get("value"), x.get("C5", {}).get("value")))
PY
}
for v in "${VARS[@]}"; do
  opt=$([ "$v" = "-" ] && echo "" || echo "$v")
  if [ -z "$NO_TRACE" ]; then
    ff=$(echo "$opt" | grep -o "FRESH_FIRST=[01]" | cut -d= -f2 || true)
    sc=$(echo "$opt" | grep -o "SCHED=[0-9]" | cut -d= -f2 || true)
    EIK_FRESH_FIRST=${ff:-0} EIK_SCHED=${sc:-1} bash tools/gpu_trace.sh > /dev/null || { echo trace failed; cat $O/trace.txt; exit 1; }
    cp $O/trace.txt "$O/${TAG}_trace_${v//[^A-Za-z0-9_]/_}.txt"; echo "trace [$v]"; grep -E "kernel|critical|busy" $O/trace.txt
  fi
done
for i in 1 2; do
  for v in "${VARS[@]}"; do
    opt=$([ "$v" = "-" ] && echo "" || echo "$v")
    f="$O/${TAG}_bench_${v//[^A-Za-z0-9_]/_}_$i.json"
    EIK_OPTIONS="$opt" timeout -k 10 300 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > "$f" 2> $O/${TAG}_bench.err || { echo "bench rc=$?"; tail -n 20 $O/${TAG}_bench.err; exit 1; }
    summ "$f" "[$v]"
  done
  [ -n "$ONCE" ] && break
done
true
