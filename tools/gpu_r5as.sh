# round 5: iterate_fit on the compact solution (no per-iteration expand / gathers) — the whole GPU
# suite, then smooth_fit end to end at C4 twice
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5as}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config c4 --e2e 3 > $OUT/e2e_$i.json 2> $OUT/e2e_$i.err || { echo "e2e failed"; tail -5 $OUT/e2e_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/e2e_$i.json').read().strip().splitlines()[-1]); t=d['timing']; print('e2e', round(d['wall_s'],3), round(t['iteration'],3), t['lsq_iters_per_solve'], round(t['edit'],3))"
done
