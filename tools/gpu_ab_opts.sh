# A/B of solver options (EIK_OPTIONS strings) on one library, alternating, 2 rounds:
#   OPTS="-|FRESH_FIRST=1" bash tools/gpu_ab_opts.sh [bench args...]     ('|'-separated; "-" = the defaults)
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
IFS='|' read -ra VARIANTS <<< "${OPTS:--}"
for i in 1 2; do
  for j in "${!VARIANTS[@]}"; do
    v="${VARIANTS[$j]}"; [ "$v" = "-" ] && v=""
    EIK_OPTIONS="$v" timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/abo_$j.json 2> $O/abo_$j.err || { echo "bench [$v] rc=$?"; tail -n 20 $O/abo_$j.err; exit 1; }
    python - "$j" "$v" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/abo_{sys.argv[1]}.json"))
r = d["roofline"]; x = d.get("extra_configs", {})
print(f"[{sys.argv[2]}] C2 %.3f ms %.2f Gcells/s visits %.0f inplace %.0f" % (d["ms_per_step"], d["value"], r["tile_visits_per_solve"], r["inplace_passes_per_solve"]),
      " | C3 %s | C4 %s | C5 %s" % (x.get("C3", {}).get("value"), x.get("C4_1gpu", {}).get("value"), x.get("C5", {}).get("value")), flush=True)
PY
  done
done
