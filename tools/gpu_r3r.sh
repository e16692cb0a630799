set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3r}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u tools/ewin_probe.py t64 t128 > $OUT/probe.log 2>&1; echo "probe rc=$?"; cat $OUT/probe.log | grep name
timeout -k 10 500 python -u tools/ewin_probe.py c3 > $OUT/probe_c3.log 2>&1; echo "c3 rc=$?"; tail -3 $OUT/probe_c3.log
