# round 4: EIK_ECOL A/B -- the W / E halo columns from a per-tile copy of the edge columns (lib_v3)
# against T's columns (lib): GPU tests on lib_v3, bench alternating, PMC traffic of both
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
EIKONAL_LIB=planning-motion_planning_amd/lib_v3/libeikonal.so timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r04j_tests_ecol.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/r04j_tests_ecol.log; exit 1; }
tail -n 1 $O/r04j_tests_ecol.log
VARIANTS="lib|;lib_v3|" REPS=3 BENCH_ARGS="--no-path --extras C3,C4_1gpu --extra-steps 3 --steps 10 --warmup 2" bash tools/gpu_ab2.sh || exit 1
for d in lib lib_v3; do
  EIKONAL_LIB=planning-motion_planning_amd/$d/libeikonal.so timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pf_$d -o f -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-path --no-timing --no-extra > $O/pf_$d.out 2>&1 || { echo "pmc fetch $d rc=$?"; exit 1; }
  EIKONAL_LIB=planning-motion_planning_amd/$d/libeikonal.so timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/pw_$d -o w -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-path --no-timing --no-extra > $O/pw_$d.out 2>&1 || { echo "pmc write $d rc=$?"; exit 1; }
  python tools/pmc_traffic.py /tmp/pf_$d /tmp/pw_$d "fim2d_persist_kernel<double" f64 > $O/r04j_pmc_traffic_$d.json 2> $O/r04j_pmc.err
  python -c "import json; d=json.load(open('$O/r04j_pmc_traffic_$d.json')); print('$d', {k: d[k] for k in d if not isinstance(d[k], (dict, list))})"
done
