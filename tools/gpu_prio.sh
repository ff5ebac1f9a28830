# Walker priority A/B (record of a rejected change): the 2D and 3D walkers built with -DEIK_WALKER_PRIO=0 / 3
# (s_setprio of the walker wave; the hook was removed from gdm.hip with the change, profiles/r02p_walker_prio_ab.log).
export TMPDIR=/tmp
for p in 0 3; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DP2_NOPROBE -DEIK_WALKER_PRIO=$p tools/path2_prof.hip -o /tmp/p2_$p || exit 1
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DP3_NOPROBE -DEIK_WALKER_PRIO=$p tools/path3_prof.hip -o /tmp/p3_$p || exit 1
done
timeout -k 10 120 python tools/dumpT.py /tmp/T.f32 > /dev/null || exit 1
for r in 1 2; do
  for p in 0 3; do
    echo "PRIO=$p 2D bench T: $(timeout -k 10 60 /tmp/p2_$p /tmp/T.f32 | grep rep | tail -1)"
    echo "PRIO=$p 3D: $(timeout -k 10 60 /tmp/p3_$p | grep padded | tail -1 | cut -c1-80)"
  done
done
