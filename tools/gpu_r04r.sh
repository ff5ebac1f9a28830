export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
EIK_ROVER_PHASES=1 timeout -k 10 300 python3 tools/dropin_probe.py > $O/r04r_dropin.log 2>&1 || { echo "rc=$?"; tail -n 20 $O/r04r_dropin.log; exit 1; }
cat $O/r04r_dropin.log | grep -v "^W"
