# round 6: C2 PMC pair (fixed harness stream), latency probe, fresh-first A/B, counter list
export TMPDIR=/tmp
R=r06g
O=gpurun_out; mkdir -p $O
source tools/pmc_pair.sh
pmc_pair C2 f64 lib C2_f64 || exit 1
pmc_pair C2 f64 lib_wl C2_f64_wline || exit 1
for g in 1 256 512; do for p in 32768 33280; do timeout -k 10 60 tools/lat_probe $g 200 $p || exit 1; done; done | tee $O/${R}_lat_probe.log
OPTS="|FRESH_FIRST=1" bash tools/gpu_ab_opts.sh --no-path --extras C4_1gpu --extra-steps 4 | tee $O/${R}_fresh_first_ab.log
timeout -k 10 60 rocprofv3 -L > $O/${R}_counters.txt 2>&1 || echo "counter list rc=$?"
grep -c . $O/${R}_counters.txt
echo ALLOK
