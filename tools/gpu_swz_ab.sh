#!/bin/bash
# LDS swizzle A/B (fim2d.hip EIK_SWZ): lib = swizzled (default build), lib_alt = EIK_SWZ=0 build
#   make -C planning-motion_planning_amd/csrc FIMFLAGS=-DEIK_SWZ=0 BUILD=../build_alt OUT=../lib_alt/libeikonal.so
# Bench A/B alternating (f64 headline and f32, with the C3/C4/C5 extras), then the SQ LDS counters
# of both builds on C2 (one --pmc pass per counter group, each its own run).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for dt in f64 f32; do
  echo "== $dt"
  VARIANTS="lib_alt|;lib|" REPS=${REPS:-3} BENCH_ARGS="--dtype $dt --extra-steps 3" bash tools/gpu_ab2.sh || exit 1
done
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-path --no-timing --no-extra"
for d in lib lib_alt; do
  for dt in f64 f32; do
    i=0
    for grp in "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      EIKONAL_LIB=planning-motion_planning_amd/$d/libeikonal.so timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d /tmp/swz_${d}_${dt}_$i -o p -- python $B --dtype $dt > $O/swz_${d}_${dt}_$i.out 2>&1 || { echo "pmc $d $dt rc=$?"; tail -5 $O/swz_${d}_${dt}_$i.out; exit 1; }
      find /tmp/swz_${d}_${dt}_$i -name "*counter_collection.csv" -exec cp {} $O/swz_${d}_${dt}_$i.csv \;
    done
  done
done
echo SWZOK
