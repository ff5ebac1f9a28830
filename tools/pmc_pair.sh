# pmc_pair CFG DTYPE LIBDIR TAG: read- and write-request counter passes (separate runs) of one config alone
# (tools/one_config.py) on planning-motion_planning_amd/LIBDIR, reduced by tools/pmc_traffic.py into
# $O/${R}_pmc_traffic_TAG.json; EIK_OPTIONS passes through.  Sourced by the tools/gpu_*.sh scripts.
pmc_pair() {
  local k="fim2d_persist_kernel<double"; [ "$2" = f32 ] && k="fim2d_persist_kernel<float"
  local c
  for c in RD WR; do
    local set="TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"; [ $c = WR ] && set="TCC_EA0_WRREQ TCC_EA0_WRREQ_64B"
    EIKONAL_LIB=planning-motion_planning_amd/$3/libeikonal.so timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv \
      -d /tmp/pmc_${4}_$c -o p -- python tools/one_config.py $1 $2 3 > $O/${R}_one_${4}_$c.json 2> $O/${R}_one_${4}_$c.err || { echo "pmc $4 $c rc=$?"; return 1; }
  done
  python tools/pmc_traffic.py /tmp/pmc_${4}_RD /tmp/pmc_${4}_WR "$k" $2 > $O/${R}_pmc_traffic_$4.json 2>> $O/${R}_pmc.err
  echo "$4: $(python -c "import json;d=json.load(open('$O/${R}_pmc_traffic_$4.json'));print(d.get('bytes_per_launch'), d.get('fetch_bytes'), d.get('write_bytes'))") $(python -c "
import json;d=json.load(open('$O/${R}_one_${4}_WR.json'));r=d.get('roofline') or {}
print('value', d['value'], 'alg', r.get('alg_bytes_per_launch', d.get('alg_bytes_per_launch')), 'visits', r.get('tile_visits_per_solve', d.get('tile_visits_per_solve')), 'passes', r.get('inplace_passes_per_solve', d.get('inplace_passes_per_solve')))")"
}
