# round 6: live DD tests (incl. the layered live split), then the shared-GPU N=2 / 8 rehearsal (C5_split live)
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dd_live.py tests/test_gpu_dd.py -v --timeout 250 --timeout-method thread > $O/r06i_dd_tests.log 2>&1
rc=$?; tail -n 3 $O/r06i_dd_tests.log; grep -E 'rank [0-9]+:' $O/r06i_dd_tests.log | head -4
[ $rc -ne 0 ] && exit 1
ROUND=r06i NS="2 8" bash tools/gpu_c4_rehearsal.sh || exit 1
echo ALLOK
