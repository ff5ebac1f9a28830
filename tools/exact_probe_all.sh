for p in c0_ c1_ c2_ c3_ c4_ c5_ c6_ c7_ c8_ c9_; do timeout -k 10 60 python -u tools/exact_probe.py fm3d_early $p || exit $?; done
for p in b0_ b1_ b2_ b3_ b4_ b5_; do timeout -k 10 60 python -u tools/exact_probe.py fmm2d_bidir $p || exit $?; done
