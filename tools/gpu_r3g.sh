set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3g}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_rz.py tests/test_gpu_band_precond.py tests/test_gpu_band.py -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1; echo "tests rc=$?"; tail -15 $OUT/tests.log
