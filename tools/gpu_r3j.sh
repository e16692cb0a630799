set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3j}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi_device.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -30 $OUT/tests.log
exit $rc
