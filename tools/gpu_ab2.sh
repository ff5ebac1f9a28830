# A/B of library builds x option sets on the bench, alternating.  VARIANTS="lib_alt|;lib|SCHED=1" (dir|EIK_OPTIONS)
export TMPDIR=/tmp
O=gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS:-lib_alt|;lib|}"
for i in $(seq 1 ${REPS:-2}); do
  for v in "${VS[@]}"; do
    d=${v%%|*}; opt=${v#*|}
    f="$O/ab2_${d}_${opt//[^A-Za-z0-9]/_}.json"
    EIKONAL_LIB=planning-motion_planning_amd/$d/libeikonal.so EIK_OPTIONS="$opt" timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$f" 2> $O/ab2.err || { echo "bench $v rc=$?"; tail -n 20 $O/ab2.err; exit 1; }
    python - "$f" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]; x = d.get("extra_configs", {})
x2 = x.get("C2_f32", {})
print("%-22s C2 %.3f ms %.2f Gc/s frac %.4f vis %.0f inpl %.0f path %.2f" % (sys.argv[2], d["ms_per_step"], d["value"], r["frac"], r["tile_visits_per_solve"], r["inplace_passes_per_solve"], d.get("ms_to_path") or 0),
      "| C3 %s | C4 %s | C5 %s | C5_f32 %s | C2_f32 %s" % (x.get("C3", {}).get("value"), x.get("C4_1gpu", {}).get("value"), x.get("C5", {}).get("value"), x.get("C5_f32", {}).get("value"), x2.get("ms_per_step")))
PY
  done
done
