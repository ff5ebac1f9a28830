# Round-end evidence on the final tree (one GPU box): GPU suite + smoke, PMC traffic of the headline, C5
# and C3 / C4 (request-size counters, tools/pmc_traffic.py), the bench line (which reads those), and the
# kernel-trace stats of the same bench command.  Outputs under gpurun_out/${ROUND}_*.
#   ROUND=r06z bash tools/gpu_final.sh
export TMPDIR=/tmp
R=${ROUND:-r06z}
O=gpurun_out; mkdir -p $O
source tools/pmc_pair.sh
if [ -z "$SKIP_TESTS" ]; then
  ROUND=$R bash tools/gpu_tests.sh || exit 1
fi
RDC="TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"; WRC="TCC_EA0_WRREQ TCC_EA0_WRREQ_64B"
for D in f64 f32; do
  K="fim2d_persist_kernel<double"; [ $D = f32 ] && K="fim2d_persist_kernel<float"
  timeout -k 10 300 rocprofv3 --pmc $RDC --kernel-trace --output-format csv -d /tmp/pf_$D -o f -- python bench.py --dtype $D --steps 3 --warmup 1 --no-cpu-baseline --no-path --no-timing --no-extra > $O/${R}_pmc_$D.out 2>&1 || { echo "pmc rd $D rc=$?"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc $WRC --kernel-trace --output-format csv -d /tmp/pw_$D -o w -- python bench.py --dtype $D --steps 3 --warmup 1 --no-cpu-baseline --no-path --no-timing --no-extra >> $O/${R}_pmc_$D.out 2>&1 || { echo "pmc wr $D rc=$?"; exit 1; }
  python tools/pmc_traffic.py /tmp/pf_$D /tmp/pw_$D "$K" $D > $O/pmc_traffic_$D.json || exit 1
done
C5="python bench.py --dtype f64 --steps 1 --warmup 0 --no-cpu-baseline --no-path --no-timing --extras C5 --extra-steps 2"
timeout -k 10 300 rocprofv3 --pmc $RDC --kernel-trace --output-format csv -d /tmp/pf_c5 -o f -- $C5 > $O/${R}_pmc_c5.out 2>&1 || { echo "pmc rd c5 rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc $WRC --kernel-trace --output-format csv -d /tmp/pw_c5 -o w -- $C5 >> $O/${R}_pmc_c5.out 2>&1 || { echo "pmc wr c5 rc=$?"; exit 1; }
python tools/pmc_traffic.py /tmp/pf_c5 /tmp/pw_c5 "fim2dl_persist_kernel<float" f32 > $O/pmc_traffic_c5.json || exit 1
python tools/pmc_traffic.py /tmp/pf_c5 /tmp/pw_c5 "fim2dl_persist_kernel<double" f64 > $O/pmc_traffic_c5_f64.json || exit 1
for c in "C3 f64 pmc_traffic_c3" "C3 f32 pmc_traffic_c3_f32" "C4 f64 pmc_traffic_c4" "C4 f32 pmc_traffic_c4_f32"; do
  set -- $c
  pmc_pair $1 $2 lib ${1}_$2 || exit 1
  cp $O/${R}_pmc_traffic_${1}_$2.json $O/$3.json
done
# the PMC summaries go where bench.py reads them, then the line and its kernel-trace stats
cp $O/pmc_traffic_*.json profiles/
timeout -k 10 600 python bench.py > $O/bench_$R.json 2> $O/bench_$R.err || { echo "bench rc=$?"; tail -n 20 $O/bench_$R.err; exit 1; }
tail -c 600 $O/bench_$R.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$R -o prof -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/${R}_prof_bench.json 2> $O/${R}_prof.err || { echo "prof rc=$?"; exit 1; }
find /tmp/prof_$R -name "*kernel_stats.csv" -exec cp {} $O/${R}_kernel_stats.csv \;
echo ALLOK
