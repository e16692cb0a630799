# round 4, session t (development): the full-size (C4) property tests
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4t}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py -v --timeout 400 --timeout-method thread --durations=5 > $OUT/gpu_tests.log 2>&1
rc=$?; tail -12 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -20
exit $rc
