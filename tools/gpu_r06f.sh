# round 6: C4 fp64 read-excess experiments (PMC pairs), then the memory-op latency probe
export TMPDIR=/tmp
R=r06f
O=gpurun_out; mkdir -p $O
pmc_pair() {  # $1 cfg $2 dtype $3 lib dir $4 tag   (EIK_OPTIONS from the environment)
  local k="fim2d_persist_kernel<double"; [ "$2" = f32 ] && k="fim2d_persist_kernel<float"
  for c in FETCH_SIZE WRITE_SIZE; do
    EIKONAL_LIB=planning-motion_planning_amd/$3/libeikonal.so timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv \
      -d /tmp/pmc_${4}_$c -o p -- python tools/one_config.py $1 $2 3 > $O/${R}_one_${4}_$c.json 2> $O/${R}_one_${4}_$c.err || { echo "pmc $4 $c rc=$?"; return 1; }
  done
  python tools/pmc_traffic.py /tmp/pmc_${4}_FETCH_SIZE /tmp/pmc_${4}_WRITE_SIZE "$k" $2 > $O/${R}_pmc_traffic_$4.json 2>> $O/${R}_pmc.err
  echo "$4: $(python -c "import json;d=json.load(open('$O/${R}_pmc_traffic_$4.json'));print(d.get('bytes_per_launch'), d.get('fetch_bytes'), d.get('write_bytes'))") $(python -c "
import json;d=json.load(open('$O/${R}_one_${4}_WRITE_SIZE.json'));r=d.get('roofline') or {}
print('value', d['value'], 'alg', r.get('alg_bytes_per_launch', d.get('alg_bytes_per_launch')), 'visits', r.get('tile_visits_per_solve', d.get('tile_visits_per_solve')), 'passes', r.get('inplace_passes_per_solve', d.get('inplace_passes_per_solve')))")"
}
EIK_OPTIONS=PRIO=0 pmc_pair C4 f64 lib C4_f64_fifo || exit 1
pmc_pair C4 f64 lib_wl C4_f64_wline || exit 1
pmc_pair C4 f64 lib C4_f64 || exit 1
pmc_pair C2 f64 lib C2_f64 || exit 1
pmc_pair C2 f64 lib_wl C2_f64_wline || exit 1
for g in 1 256 512; do for p in 32768 33280; do timeout -k 10 60 tools/lat_probe $g 200 $p || exit 1; done; done | tee $O/${R}_lat_probe.log

OPTS="|FRESH_FIRST=1" bash tools/gpu_ab_opts.sh --no-path --extras C4_1gpu --extra-steps 4 | tee $O/${R}_fresh_first_ab.log
echo ALLOK
