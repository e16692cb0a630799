set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3p}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_smooth_fit.py tests/test_gpu_mg.py tests/test_gpu_cgnr.py tests/test_gpu_lsqr.py -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAIL|Error |error:|^E |passed|failed" $OUT/tests.log | head -30
exit 0
