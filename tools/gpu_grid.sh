export TMPDIR=/tmp
O=gpurun_out
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/qprof.hip -o /tmp/qprof > $O/qprof_build.log 2>&1 || { echo build fail; cat $O/qprof_build.log; exit 1; }
timeout -k 10 120 python tools/dumpcost.py 4096 /tmp/c.f32 > /dev/null 2>&1 || { echo dump fail; exit 1; }
for g in 256 384 512 768 1024; do
  timeout -k 10 60 /tmp/qprof 4096 $g /tmp/c.f32 > $O/qg.txt 2>&1 || { echo qprof rc=$?; cat $O/qg.txt; exit 1; }
  head -1 $O/qg.txt; grep -E "sweep |grab|busy" $O/qg.txt
  timeout -k 10 60 /tmp/qprof 4096 $g > $O/qg.txt 2>&1 || { echo qprof rc=$?; exit 1; }
  head -1 $O/qg.txt; grep -E "sweep |grab|busy" $O/qg.txt
done
