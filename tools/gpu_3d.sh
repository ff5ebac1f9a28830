export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_fim3d.py -x -q > $O/t_3d.log 2>&1 || { echo "tests rc=$?"; tail -n 40 $O/t_3d.log; exit 1; }
tail -n 2 $O/t_3d.log
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-path > $O/bench_extra.json 2> $O/bench_extra.err || { echo "bench rc=$?"; tail -n 20 $O/bench_extra.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_extra.json')); print(d['value']); print(json.dumps(d['extra_configs'], indent=1))"
