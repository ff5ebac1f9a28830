export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_path.py -x -q > $O/t_path.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/t_path.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_path.json 2> $O/bench_path.err || { echo "bench rc=$?"; tail -n 20 $O/bench_path.err; exit 1; }
find /tmp/prof -name "*kernel_stats.csv" -exec cp {} $O/path_kernel_stats.csv \;
echo ALLOK
