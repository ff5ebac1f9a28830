# the round script's kernel-trace pass alone (kernel stats of the bench's headline kernel)
export TMPDIR=/tmp
R=${ROUND:-rxx}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$R -o prof -- python bench.py --steps 40 --warmup 3 --no-cpu-baseline --extras C5 --extra-steps 3 > $O/prof_$R.out 2> $O/prof_$R.err || { echo "prof rc=$?"; exit 1; }
find /tmp/prof_$R -name "*kernel_stats.csv" -exec cp {} $O/${R}_kernel_stats.csv \;
grep '^{' $O/prof_$R.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench avg_launch_us', d['roofline']['avg_launch_us'], 'ms_per_step', d['ms_per_step'])"
grep 'fim2d_persist_kernel<double, 1, false>' $O/${R}_kernel_stats.csv | cut -d, -f1-4
