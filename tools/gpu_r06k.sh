# round 6: layered live DD with bands (tests + shared rehearsal), fp32 layered 24-row tiles A/B, residency slope
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dd_live.py -v --timeout 250 --timeout-method thread -k "c5 or c4_split" > $O/r06k_dd_tests.log 2>&1
rc=$?; tail -n 2 $O/r06k_dd_tests.log; grep -E 'rank [0-9]+:' $O/r06k_dd_tests.log | head -4
[ $rc -ne 0 ] && exit 1
ROUND=r06k NS="2 8" BENCH_ARGS="--extra-steps 3" bash tools/gpu_c4_rehearsal.sh > /dev/null || exit 1
python - <<'PY'
import json
for n in (2, 8):
    L = [l for l in open(f'gpurun_out/r06k_c4_rehearsal_n{n}.log') if l.startswith('{')]
    d = json.loads(L[-1]); x = d.get('extra_configs', {}).get('C5_split', {})
    print(n, 'C4', d['value'], d['ms_per_step'], '| C5_split', {k: x.get(k) for k in ('dd_mode', 'value', 'ms_per_step', 'dd_field_ok', 'dd_rounds_per_solve', 'dd_live_error')}, x.get('dd_per_rank', {}).get('visits_vs_single_domain'))
PY
AB_TESTS="tests/test_gpu_fim3d.py" LIBS="lib lib_l24" bash tools/gpu_ab.sh --dtype f32 --no-path --extras C5 --extra-steps 5 | tee $O/r06k_l24_ab.log
bash tools/gpu_r06j.sh
