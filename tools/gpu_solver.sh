# Solver iteration on the GPU box: FIM parity tests, phase profile (qprof), bench line.
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_fim2d.py tests/test_gpu_dd.py tests/test_gpu_fim3d.py -x -q > $O/t_solver.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/t_solver.log; exit 1; }
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/qprof.hip -o /tmp/qprof > $O/qprof_build.log 2>&1 || { echo build fail; cat $O/qprof_build.log; exit 1; }
timeout -k 10 120 python tools/dumpcost.py 4096 /tmp/c.f32 > /dev/null 2>&1 || { echo dump fail; exit 1; }
timeout -k 10 60 /tmp/qprof 4096 1024 /tmp/c.f32 > $O/qprof.txt 2>&1 || { echo qprof rc=$?; cat $O/qprof.txt; exit 1; }
timeout -k 10 60 /tmp/qprof 4096 1024 >> $O/qprof.txt 2>&1 || { echo qprof2 rc=$?; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_solver.json 2> $O/bench_solver.err || { echo "bench rc=$?"; tail -n 20 $O/bench_solver.err; exit 1; }
tail -n 1 $O/t_solver.log; cat $O/qprof.txt; cat $O/bench_solver.json
