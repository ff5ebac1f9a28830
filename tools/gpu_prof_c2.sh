# Kernel-trace stats of the headline bench command alone (C2 fp64, no extra configs), for the roofline's
# duration check against the line's event average.  Outputs under gpurun_out/${ROUND}_*.
#   ROUND=r06z3 bash tools/gpu_prof_c2.sh
export TMPDIR=/tmp
R=${ROUND:-r06z3}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c2_$R -o prof -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/${R}_prof_c2_bench.json 2> $O/${R}_prof_c2.err || { echo "prof rc=$?"; exit 1; }
find /tmp/prof_c2_$R -name "*kernel_stats.csv" -exec cp {} $O/${R}_kernel_stats_c2.csv \;
grep persist $O/${R}_kernel_stats_c2.csv | cut -d, -f1-4
