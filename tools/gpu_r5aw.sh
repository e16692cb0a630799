# round 5 late: the bench line at the other BASELINE configs on the final tree (c1, c2, c3, c5)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5aw}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in c1 c2 c3 c5; do
  timeout -k 10 400 python3 bench.py --config $c --no-pmc --no-cpu > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -5 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['value']), d['unit'][:12], 'solve', d.get('solve_precond','')[:12], round(d.get('solve_time_s',0),4), d.get('solve_iters'), 'lsqr', round(d.get('lsqr_iters_per_s') or 0))"
done
