# SQ-level counters of the persistent FIM kernel on the bench raster (one --pmc pass per group,
# each its own run): LDS vs VALU occupancy of the sweep.   bash tools/gpu_pmc_sq.sh
export TMPDIR=/tmp
O=${O:-gpurun_out}
rocprofv3 -L > $O/pmc_list.txt 2>&1 || true
B=${BENCH:-"python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-path --no-timing --no-extra"}
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d /tmp/pmcsq$i -o p -- $B > $O/pmcsq$i.out 2>&1 || { echo "pmc pass $i rc=$?"; tail -5 $O/pmcsq$i.out; exit 1; }
  find /tmp/pmcsq$i -name "*counter_collection.csv" -exec cp {} $O/pmcsq$i.csv \;
done
echo PMCOK
