# round 6: compute_E windows factored in batches (LSQ_E_FBATCH) — tests, then C4 at batch 8 and 16
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6e}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_errors_window.py tests/test_gpu_band.py tests/test_gpu_smooth_fit.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/e_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/e_tests.log; exit 1; }
tail -3 $OUT/e_tests.log
timeout -k 10 400 python -u tools/compute_e_at.py c4 > $OUT/ce_c4_b8.json 2>&1 || { echo "c4 b8 failed"; tail -20 $OUT/ce_c4_b8.json; exit 1; }
tail -1 $OUT/ce_c4_b8.json | cut -c1-700
LSQ_E_FBATCH=16 timeout -k 10 400 python -u tools/compute_e_at.py c4 > $OUT/ce_c4_b16.json 2>&1 || { echo "c4 b16 failed"; tail -20 $OUT/ce_c4_b16.json; exit 1; }
tail -1 $OUT/ce_c4_b16.json | cut -c1-700
