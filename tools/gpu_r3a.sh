set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3a
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_aniso.py tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_lsqr.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
echo "rc=$?" >> $OUT/tests.log
tail -5 $OUT/tests.log
