# 3D path kernel: parity tests (3D solver, arm volumes) + per-point timing + C5 bench line
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fim3d.py tests/test_gpu_arm.py -x -q --timeout 120 --timeout-method thread > $O/p3_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/p3_tests.log; exit 1; }
tail -n 2 $O/p3_tests.log
timeout -k 10 120 python tools/path3_bench.py > $O/p3_bench.log 2>&1 || { echo "p3 rc=$?"; tail -n 20 $O/p3_bench.log; exit 1; }
cat $O/p3_bench.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/p3_benchline.json 2> $O/p3_benchline.err || { echo "bench rc=$?"; tail $O/p3_benchline.err; exit 1; }
python -c "import json; d=json.load(open('$O/p3_benchline.json')); print(d['value'], d['extra_configs']['C5'], d['extra_configs']['arm'])"
