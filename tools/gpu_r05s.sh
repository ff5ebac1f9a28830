#!/bin/bash
# round 5: event traces of the fp64 persistent kernel on the bench raster (tools/trace.hip, the
# final tree's sweep): FIFO and priority bands, the critical chain split by tools/trace_an.py
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/trace.hip -o /tmp/trace || exit 1
timeout -k 10 120 python tools/dumpcost.py 4096 /tmp/c.f32 > /dev/null 2>&1 || { echo dump fail; exit 1; }
: > $O/r05s_trace.txt
for pr in 1; do
  EIK_TRACE_F64=1 EIK_TRACE_PRIO=$pr timeout -k 10 60 /tmp/trace 4096 ${TRACE_GRID:-0} /tmp/c.f32 /tmp/tr.bin 40 >> $O/r05s_trace.txt 2>&1 || { echo "trace rc=$?"; cat $O/r05s_trace.txt; exit 1; }
  timeout -k 10 300 python tools/trace_an.py /tmp/tr.bin >> $O/r05s_trace.txt 2>&1 || { echo "an rc=$?"; cat $O/r05s_trace.txt; exit 1; }
done
cat $O/r05s_trace.txt
echo R05S_OK
