# 2D path walker: phase stamps (instrumented) and the un-instrumented time, synthetic field and bench field
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/path2_prof.hip -o /tmp/p2 && hipcc --offload-arch=gfx950 -O3 -std=c++17 -DP2_NOPROBE tools/path2_prof.hip -o /tmp/p2n || exit 1
timeout -k 10 120 python tools/dumpT.py /tmp/T.f32 || exit 1
timeout -k 10 60 /tmp/p2 | tail -5 && timeout -k 10 60 /tmp/p2n | tail -5 | head -1
timeout -k 10 60 /tmp/p2 /tmp/T.f32 | tail -5 && timeout -k 10 60 /tmp/p2n /tmp/T.f32 | tail -5 | head -1
