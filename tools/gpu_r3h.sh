set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3h}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -k "cgnr or mg" -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -30 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_aniso.py -k virtual -x -v --timeout 150 --timeout-method thread > $OUT/aniso.log 2>&1; rc=$?; echo "aniso rc=$rc"; tail -15 $OUT/aniso.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_rccl.py -x -v --timeout 300 --timeout-method thread > $OUT/rccl.log 2>&1; rc=$?; echo "rccl rc=$rc"; tail -15 $OUT/rccl.log
exit $rc
