# Phase timers of the persistent FIM kernel (tools/qprof.hip): the DEM bench raster and a uniform
# map, for the default build and, when QPROF_ALT is set, a variant built with those flags.
export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/qprof.hip -o /tmp/qprof > $O/qprof_build.log 2>&1 || { echo build fail; cat $O/qprof_build.log; exit 1; }
if [ -n "$QPROF_ALT" ]; then
  hipcc --offload-arch=gfx950 -O3 -std=c++17 $QPROF_ALT tools/qprof.hip -o /tmp/qprof_alt >> $O/qprof_build.log 2>&1 || { echo alt build fail; exit 1; }
fi
timeout -k 10 120 python tools/dumpcost.py 4096 /tmp/c.f32 > /dev/null 2>&1 || { echo dump fail; exit 1; }
: > $O/qprof.txt
for g in ${QPROF_GRIDS:-768}; do
  timeout -k 10 60 /tmp/qprof 4096 $g /tmp/c.f32 >> $O/qprof.txt 2>&1 || { echo qprof rc=$?; cat $O/qprof.txt; exit 1; }
  [ -n "$QPROF_ALT" ] && { echo "--- alt ($QPROF_ALT)" >> $O/qprof.txt; timeout -k 10 60 /tmp/qprof_alt 4096 $g /tmp/c.f32 >> $O/qprof.txt 2>&1 || { echo qprof alt rc=$?; exit 1; }; }
  timeout -k 10 60 /tmp/qprof 4096 $g - >> $O/qprof.txt 2>&1 || { echo qprof2 rc=$?; exit 1; }
done
cat $O/qprof.txt
