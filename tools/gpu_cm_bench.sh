export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pc -o p -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-path --no-timing --extra-steps 3 > gpurun_out/bcm.json 2> gpurun_out/bcm.err || { echo rc=$?; tail -n 20 gpurun_out/bcm.err; exit 1; }
find /tmp/pc -name "*kernel_stats.csv" -exec cp {} gpurun_out/cm_stats.csv \;
python -c "import json; d=json.loads(open('gpurun_out/bcm.json').read().strip().splitlines()[-1]); print(json.dumps(d['extra_configs']['costmap'], indent=1))"
grep -E "cm_|eik::" gpurun_out/cm_stats.csv | cut -c1-150 | head -30
