# One GPU-box pass of the round's evidence: GPU tests, smoke, the bench line, kernel-trace stats
# and the two PMC passes (read / write request counters in separate runs), reduced to small summaries.
#   ROUND=r03 DTYPE=f64 bash tools/gpu_round.sh      (outputs under gpurun_out/)
#   SKIP_TESTS=1 skips the GPU test suite and smoke.
export TMPDIR=/tmp
R=${ROUND:-r03}
D=${DTYPE:-f64}
K=$([ "$D" = f64 ] && echo "fim2d_persist_kernel<double" || echo "fim2d_persist_kernel<float")
O=gpurun_out
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/t_all.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/t_all.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
fi
timeout -k 10 600 python bench.py --dtype $D > $O/bench_$R.json 2> $O/bench_$R.err || { echo "bench rc=$?"; tail -n 20 $O/bench_$R.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$R -o prof -- python bench.py --dtype $D --steps 40 --warmup 3 --no-cpu-baseline --extras C5 --extra-steps 3 > $O/prof_$R.out 2> $O/prof_$R.err || { echo "prof rc=$?"; exit 1; }
find /tmp/prof_$R -name "*kernel_stats.csv" -exec cp {} $O/${R}_kernel_stats.csv \;
# memory-side bytes from the L2's request counters by size (tools/pmc_traffic.py): reads, then writes
RDC="TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"; WRC="TCC_EA0_WRREQ TCC_EA0_WRREQ_64B"
timeout -k 10 300 rocprofv3 --pmc $RDC --kernel-trace --output-format csv -d /tmp/pmc_fetch_$R -o f -- python bench.py --dtype $D --steps 3 --warmup 1 --no-cpu-baseline --no-path --no-timing --no-extra > $O/pmc_fetch.out 2> $O/pmc_fetch.err || { echo "pmc fetch rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc $WRC --kernel-trace --output-format csv -d /tmp/pmc_write_$R -o w -- python bench.py --dtype $D --steps 3 --warmup 1 --no-cpu-baseline --no-path --no-timing --no-extra > $O/pmc_write.out 2> $O/pmc_write.err || { echo "pmc write rc=$?"; exit 1; }
python tools/pmc_traffic.py /tmp/pmc_fetch_$R /tmp/pmc_write_$R "$K" $D > $O/pmc_traffic_${R}_$D.json 2> $O/pmc_traffic.err
# the layered solver (C5, fim2dl_persist_kernel) in its own pair of passes
C5="python bench.py --dtype $D --steps 1 --warmup 0 --no-cpu-baseline --no-path --no-timing --extras C5 --extra-steps 2"
timeout -k 10 300 rocprofv3 --pmc $RDC --kernel-trace --output-format csv -d /tmp/pmc_fetch_c5_$R -o f -- $C5 > $O/pmc_fetch_c5.out 2>&1 || { echo "pmc fetch c5 rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc $WRC --kernel-trace --output-format csv -d /tmp/pmc_write_c5_$R -o w -- $C5 > $O/pmc_write_c5.out 2>&1 || { echo "pmc write c5 rc=$?"; exit 1; }
# (a --dtype f64 run holds both C5 kernels: the fp64 one (C5) and the fp32 one (C5_f32))
python tools/pmc_traffic.py /tmp/pmc_fetch_c5_$R /tmp/pmc_write_c5_$R "fim2dl_persist_kernel<float" f32 > $O/pmc_traffic_${R}_c5.json 2>> $O/pmc_traffic.err
if [ "$D" = f64 ]; then
python tools/pmc_traffic.py /tmp/pmc_fetch_c5_$R /tmp/pmc_write_c5_$R "fim2dl_persist_kernel<double" f64 > $O/pmc_traffic_${R}_c5_f64.json 2>> $O/pmc_traffic.err
fi
echo ALLOK
