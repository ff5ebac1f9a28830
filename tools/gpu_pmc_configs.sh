# PMC traffic (FETCH_SIZE / WRITE_SIZE in separate passes) of the throughput configs' solver launches,
# each config alone (tools/one_config.py), reduced by tools/pmc_traffic.py; then the queue counters of
# an EIK_QDEBUG build (tools/qcount_probe.py) and the same PMC pair on a build with a longer poll
# backoff (lib_sl: EIK_PRIO_SLEEP=32), for the attribution of the bytes above the algorithmic ones.
#   ROUND=r06e CONFIGS="C3 C4" DTYPES="f64 f32" bash tools/gpu_pmc_configs.sh
export TMPDIR=/tmp
R=${ROUND:-r06e}
O=gpurun_out; mkdir -p $O
pmc_pair() {  # $1 cfg $2 dtype $3 lib dir $4 tag
  local k="fim2d_persist_kernel<double"; [ "$2" = f32 ] && k="fim2d_persist_kernel<float"
  for c in FETCH_SIZE WRITE_SIZE; do
    EIKONAL_LIB=planning-motion_planning_amd/$3/libeikonal.so timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv \
      -d /tmp/pmc_${4}_$c -o p -- python tools/one_config.py $1 $2 3 > $O/${R}_one_${4}_$c.json 2> $O/${R}_one_${4}_$c.err || { echo "pmc $4 $c rc=$?"; return 1; }
  done
  python tools/pmc_traffic.py /tmp/pmc_${4}_FETCH_SIZE /tmp/pmc_${4}_WRITE_SIZE "$k" $2 > $O/${R}_pmc_traffic_$4.json 2>> $O/${R}_pmc.err
  echo "$4: $(python -c "import json;d=json.load(open('$O/${R}_pmc_traffic_$4.json'));print(d.get('bytes_per_launch'), d.get('fetch_bytes'), d.get('write_bytes'))") value $(python -c "import json;d=json.load(open('$O/${R}_one_${4}_WRITE_SIZE.json'));print(d['value'], d['roofline']['alg_bytes_per_launch'])")"
}
for cfg in ${CONFIGS:-C3 C4}; do for dt in ${DTYPES:-f64 f32}; do
  pmc_pair $cfg $dt lib ${cfg}_$dt || exit 1
done; done
for cfg in C4 C3; do
  EIKONAL_LIB=planning-motion_planning_amd/lib_qd/libeikonal.so timeout -k 10 300 python tools/qcount_probe.py $cfg f64 2 > $O/${R}_qcount_$cfg.json 2> $O/${R}_qcount_$cfg.err || { echo "qcount $cfg rc=$?"; exit 1; }
  cat $O/${R}_qcount_$cfg.json
done
pmc_pair C4 f64 lib_sl C4_f64_sleep32 || exit 1
echo ALLOK
