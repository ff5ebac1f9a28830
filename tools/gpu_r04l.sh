# round 4: timeline of planner step 1 (kernels + copies of one eik_rover_path_f64 call)
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
OPTS_LIST="" ROVER_ONLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r04l -o tl -- python3 tools/rover_probe.py > $O/r04l_rover.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r04l_rover.log; exit 1; }
python3 tools/timeline.py /tmp/r04l > $O/r04l_timeline.txt 2>&1 || { echo "timeline rc=$?"; tail -n 20 $O/r04l_timeline.txt; }
grep -E "^default" $O/r04l_rover.log
tail -n 60 $O/r04l_timeline.txt
