# round 4, closing (development): the other BASELINE configurations on the committed code —
# C1, C2 (2-D), C3, C5 (2048²×12, 8 M points, isotropic) — block-Jacobi it/s and the full solves
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4cfg}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in c1 c2 c3 c5; do
  timeout -k 10 400 python3 bench.py --config $cfg --no-cpu --no-pmc --steps 100 --warmup 10 > $OUT/$cfg.json 2> $OUT/$cfg.err || { echo "$cfg failed"; tail -3 $OUT/$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$cfg.json')); bj=d.get('solve_block_jacobi', {}); print('$cfg', round(d['value']), 'solve', round(d['solve_time_s'],4), d['solve_iters'], d.get('solve_precond'), 'setup', round(d.get('solve_setup_s',0)*1e3,2), 'BJ', bj.get('solve_iters'), round(bj.get('solve_time_s',0),4), 'form', round(d['device_formation_s'],3), 'dev_GB', round(d['config'].get('rank0_system', d['config'].get('system', {})).get('device_bytes', 0)/1e9, 2))"
done
