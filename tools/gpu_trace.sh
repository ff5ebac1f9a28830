# Event traces of the persistent FIM kernel (tools/trace.hip) on the DEM bench raster and a
# uniform map, analysed by tools/trace_an.py.
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 python tools/dumpcost.py 4096 /tmp/c.f32 > /dev/null 2>&1 || { echo dump fail; exit 1; }
: > $O/trace.txt
for g in ${TRACE_GRIDS:-768}; do
  timeout -k 10 60 tools/trace 4096 $g /tmp/c.f32 /tmp/tr_dem.bin ${TRACE_PASSES:-24} >> $O/trace.txt 2>&1 || { echo trace rc=$?; cat $O/trace.txt; exit 1; }
  timeout -k 10 300 python tools/trace_an.py /tmp/tr_dem.bin >> $O/trace.txt 2>&1 || { echo an rc=$?; cat $O/trace.txt; exit 1; }
  timeout -k 10 60 tools/trace 4096 $g - /tmp/tr_uni.bin ${TRACE_PASSES:-24} >> $O/trace.txt 2>&1 || { echo trace2 rc=$?; cat $O/trace.txt; exit 1; }
  timeout -k 10 300 python tools/trace_an.py /tmp/tr_uni.bin >> $O/trace.txt 2>&1 || { echo an2 rc=$?; cat $O/trace.txt; exit 1; }
done
cat $O/trace.txt
