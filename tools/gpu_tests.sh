# the GPU test suite + smoke on the current tree (outputs: gpurun_out/${ROUND}_gpu_tests.log, ${ROUND}_smoke.log)
export TMPDIR=/tmp
R=${ROUND:-rxx}
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/${R}_gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -n 30 $O/${R}_gpu_tests.log; exit 1; }
tail -n 1 $O/${R}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${R}_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -n 20 $O/${R}_smoke.log; exit 1; }
echo ALLOK
