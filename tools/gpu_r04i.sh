# round 4: the activation cap's cost on the uncapped solves (lib: EIK_TCAP on, lib_v2: compiled out),
# C2 fp64 + C3 + C4 alternating; then the bounded join's and capped fronts' kernels on planner step 1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
VARIANTS="lib_v2|;lib|" REPS=3 BENCH_ARGS="--no-path --extras C3,C4_1gpu --extra-steps 3 --steps 10 --warmup 2" bash tools/gpu_ab2.sh || exit 1
OPTS_LIST="FRONTS_CAP=1.1,FRONTS_CAP=1.25,FRONTS_CAP=1.1,FRONTS_CAP=1.25,FRONTS_CAP=1.5" timeout -k 10 300 python3 tools/rover_probe.py > $O/r04i_margin.log 2>&1 || { echo "margin rc=$?"; tail -n 20 $O/r04i_margin.log; exit 1; }
grep -E "^FRONTS" $O/r04i_margin.log
OPTS_LIST="," timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r04i_prof -o rover -- python3 tools/rover_probe.py > $O/r04i_rover.log 2>&1 || { echo "rover rc=$?"; tail -n 20 $O/r04i_rover.log; exit 1; }
f=$(find /tmp/r04i_prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/r04i_rover_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04i_rover_kernel_stats.csv")))
for r in rows:
    n = r["Name"]
    if any(k in n for k in ("join", "scatter_rank", "rocprim", "bidir", "fim2d_persist", "gdm2d", "cost", "cap_clean", "fronts")):
        print(f"{n[:100]:100s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:9.1f} us  total {float(r['TotalDurationNs'])/1e6:8.3f} ms")
PY
