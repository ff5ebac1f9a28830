# round 6: GPU suite on the new library, the band-ring probe on both libraries, then the bench A/B
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
ROUND=r06c bash tools/gpu_tests.sh || exit 1
for lib in lib_alt lib; do
  EIKONAL_LIB=planning-motion_planning_amd/$lib/libeikonal.so timeout -k 10 600 python -u tools/ring_probe.py 512 256 128 64 >> $O/r06c_ring_probe.log 2>&1
  rc=$?; echo "ring probe $lib rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 $O/r06c_ring_probe.log; exit 1; fi
done
grep ring $O/r06c_ring_probe.log
LIBS="lib_alt lib" bash tools/gpu_ab.sh --no-path --extras C4_1gpu --extra-steps 4
