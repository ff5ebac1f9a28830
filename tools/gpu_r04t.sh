# capped fronts: coarse raster side (EIK_FRONTS_COARSE 512 = F 8 at 4096^2, 256 = F 16, 1024 = F 4), planner step 1 phases
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for cs in 512 256 1024 512 256; do
  EIK_FRONTS_COARSE=$cs EIK_ROVER_PHASES=1 OPTS_LIST="" ROVER_ONLY=1 timeout -k 10 300 python3 tools/rover_probe.py > $O/r04t_$cs.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r04t_$cs.log; exit 1; }
  echo "coarse side $cs: $(grep fronts $O/r04t_$cs.log | tail -n 3 | awk '{print $3}' | tr '\n' ' ') | $(grep default $O/r04t_$cs.log)"
done
