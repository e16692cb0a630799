# round 4 (development): smooth_fit GPU tests after the one-temporary convergence check
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4sf}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_smooth_fit.py tests/test_gpu_multi_device.py tests/test_gpu_band.py -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --config c4 --e2e 3 > $OUT/e2e_c4.json 2> $OUT/e2e_c4.err || { echo "e2e failed"; tail -3 $OUT/e2e_c4.err; exit 1; }
cat $OUT/e2e_c4.json
