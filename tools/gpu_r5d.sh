# round 5 (development): compute_E windows sweeping only their interior tiles — the window /
# band tests, then compute_E at C4 (round 4: 477 s)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5d}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_errors_window.py tests/test_gpu_band.py tests/test_gpu_smooth_fit.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python3 -u tools/compute_e_at.py c4 > $OUT/compute_e_c4.json 2> $OUT/compute_e_c4.err || { echo "compute_E failed"; tail -5 $OUT/compute_e_c4.err; exit 1; }
tail -1 $OUT/compute_e_c4.json
