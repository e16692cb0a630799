# round 5 (development): pipelined compute_E windows — the error-propagation tests, then compute_E
# at C4 with 64- and 32-node tiles (lanes 3)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5g}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_errors_window.py tests/test_gpu_smooth_fit.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
for t in 64 32; do
  LSQ_E_TILE=$t timeout -k 10 500 python3 -u tools/compute_e_at.py c4 > $OUT/compute_e_c4_t$t.json 2> $OUT/compute_e_c4_t$t.err || { echo "compute_E t=$t failed"; tail -5 $OUT/compute_e_c4_t$t.err; exit 1; }
  tail -1 $OUT/compute_e_c4_t$t.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('t=$t', round(d['wall_s'],1), d['timing']['E_window'])"
done
