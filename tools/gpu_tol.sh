export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/qprof.hip -o /tmp/qprof > $O/qprof_build.log 2>&1 || { echo build fail; cat $O/qprof_build.log; exit 1; }
timeout -k 10 120 python tools/dumpcost.py 4096 /tmp/c.f32 > /dev/null 2>&1 || { echo dump fail; exit 1; }
for t in 0 1e-7 3e-7 1e-6 3e-6 1e-5; do
  timeout -k 10 60 /tmp/qprof 4096 768 /tmp/c.f32 1 $t > $O/qg.txt 2>&1 || { echo qprof rc=$?; cat $O/qg.txt; exit 1; }
  head -1 $O/qg.txt
  timeout -k 10 60 /tmp/qprof 4096 768 - 1 $t > $O/qg.txt 2>&1 || { echo qprof rc=$?; exit 1; }
  head -1 $O/qg.txt
done
