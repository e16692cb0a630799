# Round-3 closing evidence for the committed state: the whole -m gpu suite, then smoke, the default
# bench line, rocprof kernel stats, C5a and one rank's window at N = 8 (tools/gpu_r3s2e.sh)
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3s2h}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/gpu_r3s2e.sh ${1:-r3s2h}
