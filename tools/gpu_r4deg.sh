# round 4 (development): smoothing degrees at C5a (anisotropic: the weak multigrid case) and C4 —
# level 0 (LSQ_MG_DEG0, symmetric) and the coarse levels (LSQ_MG_DEG)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4deg}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in c5a c4; do
for v in "LSQ_MG_DEG0=2" "LSQ_MG_DEG0=3" "LSQ_MG_DEG0=1" "LSQ_MG_DEG=2" "LSQ_MG_DEG0=3 LSQ_MG_DEG=2"; do
  tag=${cfg}_$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-pmc --steps 20 --warmup 5 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$cfg $v', 'MG', round(d['solve_time_s'],4), d['solve_iters'], round(d['solve_time_s']/d['solve_iters']*1e3,2), 'ms/it setup', round(d['solve_setup_s']*1e3,1))"
done
done
