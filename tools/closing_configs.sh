# round 6 closing: the bench on the other BASELINE configurations and the per-rank windows (committed tree)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6u
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in c1 c2 c3 c5; do
  timeout -k 10 600 python3 bench.py --config $c --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/$c.json 2> $OUT/$c.err || { echo "$c failed"; tail -5 $OUT/$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$c.json').read().strip().splitlines()[-1]); print('$c', round(d['value']), round(d['ms_per_step'],4), 'solve', d.get('solve_method'), d.get('solve_precond'), d.get('solve_time_s'), d.get('solve_iters'), 'lsqr', round(d.get('lsqr_iters_per_s') or 0))"
done
for c in c4y8 c4y4 c5y8; do
  timeout -k 10 300 python3 bench.py --config $c --dist --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/$c.json 2> $OUT/$c.err || { echo "$c failed"; tail -5 $OUT/$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$c.json').read().strip().splitlines()[-1]); print('$c', round(d['value']), round(d['ms_per_step'],4), 'MG', d.get('solve_time_s'), d.get('solve_iters'))"
done
