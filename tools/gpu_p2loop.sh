# 2D path walker A/B: the single-exit loop (FUSED=1, default) vs the plain one (FUSED=0), the
# un-instrumented kernel time on a smooth synthetic field and on the bench field.
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DP2_NOPROBE tools/path2_prof.hip -o /tmp/p2n || exit 1
timeout -k 10 120 python tools/dumpT.py /tmp/T.f32 > /dev/null || exit 1
for r in 1 2; do
  for sp in ${FORMS:-0 1 2}; do
    echo "FUSED=$sp synthetic: $(FUSED=$sp timeout -k 10 60 /tmp/p2n | grep rep | tail -1)"
    echo "FUSED=$sp bench T:   $(FUSED=$sp timeout -k 10 60 /tmp/p2n /tmp/T.f32 | grep rep | tail -1)"
  done
done
