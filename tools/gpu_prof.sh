export TMPDIR=/tmp
O=gpurun_out
R=r01
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$R -o prof -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra > $O/prof_$R.out 2> $O/prof_$R.err || { echo "prof rc=$?"; exit 1; }
find /tmp/prof_$R -name "*kernel_stats.csv" -exec cp {} $O/${R}_kernel_stats.csv \;
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_x -o prof -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-path --no-timing --extra-steps 5 > $O/prof_extra_$R.out 2> $O/prof_extra_$R.err || { echo "prof2 rc=$?"; exit 1; }
find /tmp/prof_x -name "*kernel_stats.csv" -exec cp {} $O/${R}_extra_kernel_stats.csv \;
echo ALLOK
