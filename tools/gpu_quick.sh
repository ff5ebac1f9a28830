# Quick GPU pass: a test subset (TESTS, default the 2D solver tests) then the bench without extras.
#   TESTS="tests/test_gpu_fim2d.py" ROUND=r03b bash tools/gpu_quick.sh
export TMPDIR=/tmp
R=${ROUND:-r03q}
T=${TESTS:-tests/test_gpu_fim2d.py}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > $O/${R}_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/${R}_tests.log; exit 1; }
tail -n 3 $O/${R}_tests.log
for d in ${DTYPES:-f64 f32}; do
timeout -k 10 300 python bench.py --dtype $d --no-extra --no-cpu-baseline ${BENCH_ARGS} > $O/${R}_bench_$d.json 2> $O/${R}_bench_$d.err || { echo "bench rc=$?"; tail -n 20 $O/${R}_bench_$d.err; exit 1; }
python -c "import json,sys; d=json.load(open('$O/${R}_bench_$d.json')); print('$d', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['tile_visits_per_solve'], d['roofline']['inplace_passes_per_solve'], d.get('ms_to_path'))"
done
