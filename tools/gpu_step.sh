# Product sweep-step microbenchmark for build variants: STEP_VARIANTS="name:flags;name:flags"
export TMPDIR=/tmp
O=gpurun_out
: > $O/step.txt
IFS=';' read -ra VS <<< "${STEP_VARIANTS:-default:}"
for v in "${VS[@]}"; do
  n=${v%%:*}; f=${v#*:}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 $f tools/step_bench.hip -o /tmp/step_$n >> $O/step_build.log 2>&1 || { echo "build $n failed"; tail $O/step_build.log; exit 1; }
  echo "--- $n ($f)" >> $O/step.txt
  timeout -k 10 60 /tmp/step_$n >> $O/step.txt 2>&1 || { echo "run $n rc=$?"; cat $O/step.txt; exit 1; }
done
cat $O/step.txt
