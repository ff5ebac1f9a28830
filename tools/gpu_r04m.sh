# round 4: cost-raster builder -- segment-scan disk morphology + deduplicated CCL border unions: parity
# (costmap / planner / drop-in tests), the costmap extra line, and planner step 1's timeline
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_costmap.py tests/test_gpu_planner.py tests/test_dropin.py tests/test_gpu_bidir_join.py > $O/r04m_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r04m_tests.log; exit 1; }
tail -n 1 $O/r04m_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-path --steps 3 --warmup 1 --extras costmap > $O/r04m_bench.json 2> $O/r04m_bench.err || { echo "bench rc=$?"; tail -n 20 $O/r04m_bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/r04m_bench.json'))['extra_configs']['costmap']; print('costmap', d['ms_per_step'], 'ms', d['value'], 'Gcells/s; planner step 1', d['planner_step1']['ms'], 'ms')"
bash tools/gpu_r04l.sh
