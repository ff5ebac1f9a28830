#!/bin/bash
# round 5: rooflines of the throughput-bound configs -- PMC traffic pairs (FETCH_SIZE / WRITE_SIZE,
# separate runs) of C3 and C4 at one GPU in both dtypes (tools/one_config.py: only that config's
# launches), SQ counters of C3 fp64 and of the fp32 layered C5 kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for cfg in C3 C4; do
  for dt in f64 f32; do
    n=$([ $cfg = C4 ] && echo 2 || echo 3)
    k=$([ $dt = f64 ] && echo "fim2d_persist_kernel<double" || echo "fim2d_persist_kernel<float")
    sfx=$([ $dt = f64 ] && echo "" || echo "_f32")
    lc=$(echo $cfg | tr C c)
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pf_$cfg$dt -o f -- python tools/one_config.py $cfg $dt $n > /tmp/pf_$cfg$dt.out 2>&1 || { echo "fetch $cfg $dt rc=$?"; tail -5 /tmp/pf_$cfg$dt.out; exit 1; }
    timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/pw_$cfg$dt -o w -- python tools/one_config.py $cfg $dt $n > /tmp/pw_$cfg$dt.out 2>&1 || { echo "write $cfg $dt rc=$?"; tail -5 /tmp/pw_$cfg$dt.out; exit 1; }
    python tools/pmc_traffic.py /tmp/pf_$cfg$dt /tmp/pw_$cfg$dt "$k" $dt > $O/pmc_traffic_$lc$sfx.json || exit 1
    grep "^{" /tmp/pf_$cfg$dt.out | tail -1 > $O/one_${cfg}_$dt.json
    echo "$cfg $dt: $(python -c "import json;d=json.load(open('$O/pmc_traffic_$lc$sfx.json'));print(d['bytes_per_launch'], d['dispatches'])")"
  done
done
BENCH="python tools/one_config.py C3 f64 2" O=/tmp bash tools/gpu_pmc_sq.sh || exit 1
python tools/sq_summary.py /tmp/pmcsq1.csv /tmp/pmcsq2.csv --kernel "fim2d_persist_kernel<double" --label "C3 fp64 (tools/one_config.py C3 f64 2)" > $O/sq_c3_f64.json || exit 1
BENCH="python bench.py --dtype f32 --steps 1 --warmup 0 --no-cpu-baseline --no-path --no-timing --extras C5 --extra-steps 2" O=/tmp bash tools/gpu_pmc_sq.sh || exit 1
python tools/sq_summary.py /tmp/pmcsq1.csv /tmp/pmcsq2.csv --kernel "fim2dl_persist_kernel<float" --label "C5 fp32 layered" > $O/sq_c5_f32.json || exit 1
# the layered kernels' traffic on the layer-planar copies (EIK_OPT_LAYER_PLANAR=1)
C5="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-path --no-timing --extras C5 --extra-steps 2"
EIK_OPTIONS=LAYER_PLANAR=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pfp_c5 -o f -- $C5 > /tmp/pfp_c5.out 2>&1 || { echo "planar fetch rc=$?"; exit 1; }
EIK_OPTIONS=LAYER_PLANAR=1 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/pwp_c5 -o w -- $C5 > /tmp/pwp_c5.out 2>&1 || { echo "planar write rc=$?"; exit 1; }
python tools/pmc_traffic.py /tmp/pfp_c5 /tmp/pwp_c5 "fim2dl_persist_kernel<float" f32 > $O/pmc_traffic_c5_planar.json || exit 1
python tools/pmc_traffic.py /tmp/pfp_c5 /tmp/pwp_c5 "fim2dl_persist_kernel<double" f64 > $O/pmc_traffic_c5_f64_planar.json || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pf_c5 -o f -- $C5 > /tmp/pf_c5.out 2>&1 || { echo "fetch c5 rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/pw_c5 -o w -- $C5 > /tmp/pw_c5.out 2>&1 || { echo "write c5 rc=$?"; exit 1; }
python tools/pmc_traffic.py /tmp/pf_c5 /tmp/pw_c5 "fim2dl_persist_kernel<float" f32 > $O/pmc_traffic_c5_r05.json || exit 1
python tools/pmc_traffic.py /tmp/pf_c5 /tmp/pw_c5 "fim2dl_persist_kernel<double" f64 > $O/pmc_traffic_c5_f64_r05.json || exit 1
echo R05C_OK
