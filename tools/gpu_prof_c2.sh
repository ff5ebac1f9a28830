export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r06z2 -o prof -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --extras C5 --extra-steps 3 > $O/r06z2_prof_bench.json 2> $O/r06z2_prof.err || { echo "prof rc=$?"; exit 1; }
find /tmp/prof_r06z2 -name "*kernel_stats.csv" -exec cp {} $O/r06z2_kernel_stats.csv \;
grep persist $O/r06z2_kernel_stats.csv | cut -d, -f1-4
