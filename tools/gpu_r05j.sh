#!/bin/bash
# round 5: the whole GPU suite with the priority bands on by default, smoke, then the default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/r05j_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error|error" $O/r05j_tests.log | head -20; tail -30 $O/r05j_tests.log; exit 1; }
tail -1 $O/r05j_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05j_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/r05j_smoke.log; exit 1; }
tail -1 $O/r05j_smoke.log
timeout -k 10 600 python bench.py > $O/r05j_bench.json 2> $O/r05j_bench.err || { echo "bench rc=$?"; tail -20 $O/r05j_bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/r05j_bench.json')); x=d['extra_configs']
print('C2', d['value'], d['ms_per_step'], 'frac', d['roofline']['frac'])
for k,v in x.items(): print(k, v.get('value'), v.get('ms_per_step'), (v.get('roofline') or {}).get('frac'))
print('ms_to_path', d.get('ms_to_path'), 'cpu', d['cpu_baseline']['value'])"
