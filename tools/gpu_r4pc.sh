# round 4 (development): the concurrent power-step test
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4pc}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mg.py -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
