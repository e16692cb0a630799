# round 4, session d (development): C5a multigrid iteration counts of the round-3 commits (the
# 61 -> 72 regression) and of the current build's normal-operator / data-row variants
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4d}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in cf1e74e 33d1d38 5ce97ea 708e2d2 c74d764 fe9309c 86239f2 4a2b8fc; do
  (cd tools/ab/bisect/$c && timeout -k 10 240 python3 bench.py --config c5a --no-cpu --no-pmc --steps 20 --warmup 5 > $OUT/c5a_$c.json 2> $OUT/c5a_$c.err) || { echo "c5a $c failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5a_$c.json')); print('c5a $c MG', d['solve_iters'], round(d['solve_time_s'],3), 'BJ', d.get('solve_block_jacobi',{}).get('solve_iters'))"
done
for v in "LSQ_CG_RW=0" "LSQ_CG_RW_KT=0" "LSQ_CG_DMF=0"; do
  env $v timeout -k 10 240 python3 bench.py --config c5a --no-cpu --no-pmc --steps 20 --warmup 5 > $OUT/c5a_$v.json 2> $OUT/c5a_$v.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/c5a_$v.json')); print('c5a $v MG', d['solve_iters'], round(d['solve_time_s'],3), 'BJ', d['solve_block_jacobi']['solve_iters'])"
done
