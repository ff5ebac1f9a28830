# round 4: planner step 1 phase times (EIK_ROVER_PHASES=1: a synchronisation after each phase)
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
EIK_ROVER_PHASES=1 OPTS_LIST="" ROVER_ONLY=1 timeout -k 10 300 python3 tools/rover_probe.py > $O/r04n_phases.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r04n_phases.log; exit 1; }
OPTS_LIST="" ROVER_ONLY=1 FRESH=1 timeout -k 10 300 python3 tools/rover_probe.py >> $O/r04n_phases.log 2>&1 || { echo "rc=$?"; exit 1; }
grep -E "rover|default" $O/r04n_phases.log | tail -n 24
