#!/bin/bash
# round 5: 2D walker loop forms 3 (divisions from the square roots' reciprocals, gdm.hip div_rs)
# and 4 (form 3 on lane pairs: x on even lanes, y on odd):
# the exactness self-test and the loop-form bit-identity tests, the un-instrumented kernel A/B
# (forms 2 / 3, synthetic and bench fields), the s_memtime phase breakdown of both forms, and
# the bench's path line with each form.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_path.py -x -v --timeout 120 --timeout-method thread -k "fast_math or loop_forms" > $O/r05k_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/r05k_tests.log; exit 1; }
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DP2_NOPROBE tools/path2_prof.hip -o /tmp/p2n || exit 1
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/path2_prof.hip -o /tmp/p2p || exit 1
timeout -k 10 120 python tools/dumpT.py /tmp/T.f32 > /dev/null || exit 1
{
for r in 1 2 3; do
  for sp in 2 3 4; do
    echo "FUSED=$sp synthetic: $(FUSED=$sp timeout -k 10 60 /tmp/p2n | grep rep | tail -1)"
    echo "FUSED=$sp bench T:   $(FUSED=$sp timeout -k 10 60 /tmp/p2n /tmp/T.f32 | grep rep | tail -1)"
  done
done
echo "# s_memtime phase breakdown (probe build; the probes add their own cycles)"
for sp in 2 4; do
  echo "FUSED=$sp bench T (probes):"; FUSED=$sp timeout -k 10 60 /tmp/p2p /tmp/T.f32 | tail -5
done
} > $O/r05k_walker_ab.log 2>&1 || { echo "walker ab rc=$?"; tail $O/r05k_walker_ab.log; exit 1; }
for f in 2 4 2 4; do
  EIK_OPTIONS=PATH_LOOP=$f timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > /tmp/b$f.json 2> /tmp/b$f.err || { echo "bench rc=$?"; tail /tmp/b$f.err; exit 1; }
  python -c "import json;d=json.load(open('/tmp/b$f.json'));print('PATH_LOOP=$f', 'path_kernel_ms', d['path_kernel_ms'], 'us/step', d['path_us_per_step'], 'points', d['path_points'], 'ms_to_path', d['ms_to_path'])" >> $O/r05k_walker_ab.log
done
cat $O/r05k_walker_ab.log
echo R05K_OK
