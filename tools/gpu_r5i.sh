# round 5: release_full_csr test, then the full GPU suite and smoke on the committed tree
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5i}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_solve_sequence.py > $OUT/seq.log 2>&1 || { echo "sequence tests failed"; tail -30 $OUT/seq.log; exit 1; }
tail -3 $OUT/seq.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { echo "gpu suite failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
