# round 6: raw TCC request-size counters of the solver launches (C2 / C4 fp64, C4 on the FIFO)
export TMPDIR=/tmp
R=r06h
O=gpurun_out; mkdir -p $O
raw() {  # $1 cfg $2 tag (EIK_OPTIONS passes through)
  local i=0
  for set in "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ" "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_RDREQ_DRAM TCC_EA0_RD_UNCACHED_32B" "TCC_ATOMIC TCC_EA0_ATOMIC TCC_HIT TCC_MISS"; do
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d /tmp/raw_${2}_$i -o p -- python tools/one_config.py $1 f64 3 > $O/${R}_raw_${2}_$i.json 2> $O/${R}_raw_${2}_$i.err || { echo "raw $2 $i rc=$?"; tail -3 $O/${R}_raw_${2}_$i.err; return 1; }
  done
  python tools/pmc_raw.py "fim2d_persist_kernel<double" /tmp/raw_${2}_1 /tmp/raw_${2}_2 /tmp/raw_${2}_3 > $O/${R}_raw_$2.json
  python -c "import json;d=json.load(open('$O/${R}_raw_$2.json'));print('$2', 'read', d.get('read_bytes'), 'write', d.get('write_bytes'), {k: round(v) for k, v in d['per_launch'].items()})"
  python -c "import json;d=json.load(open('$O/${R}_raw_${2}_1.json'));r=d.get('roofline') or {};print('   value', d['value'], 'alg', r.get('alg_bytes_per_launch', d.get('alg_bytes_per_launch')), 'visits', r.get('tile_visits_per_solve', d.get('tile_visits_per_solve')), 'passes', r.get('inplace_passes_per_solve', d.get('inplace_passes_per_solve')))"
}
raw C2 C2 || exit 1
raw C4 C4 || exit 1
EIK_OPTIONS=PRIO=0 raw C4 C4_fifo || exit 1
echo ALLOK
