export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/qprof.hip -o /tmp/qprof > $O/qprof_build.log 2>&1 || { echo build fail; cat $O/qprof_build.log; exit 1; }
timeout -k 10 120 python tools/dumpcost.py 4096 /tmp/c.f32 > /dev/null 2>&1 || { echo dump fail; exit 1; }
timeout -k 10 60 /tmp/qprof 4096 1024 /tmp/c.f32 > $O/qprof.txt 2>&1 || { echo qprof rc=$?; cat $O/qprof.txt; exit 1; }
timeout -k 10 60 /tmp/qprof 4096 1024 >> $O/qprof.txt 2>&1 || { echo qprof2 rc=$?; exit 1; }
cat $O/qprof.txt
