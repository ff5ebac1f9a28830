export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/qprof.hip -o /tmp/qprof > $O/qprof_build.log 2>&1 || { echo build fail; tail $O/qprof_build.log; exit 1; }
timeout -k 10 180 python tools/dumpcost.py 16384 /tmp/c16.f32 > /dev/null 2>&1 || { echo dump fail; exit 1; }
timeout -k 10 120 /tmp/qprof 16384 768 /tmp/c16.f32 > $O/qprof16.txt 2>&1 || { echo qprof rc=$?; cat $O/qprof16.txt; exit 1; }
timeout -k 10 120 /tmp/qprof 16384 768 - >> $O/qprof16.txt 2>&1 || { echo qprof2 rc=$?; exit 1; }
cat $O/qprof16.txt
