# wave-strip gate A/B, small systems (development): C1 non-live role times, C1 / C3 multigrid
# solves and one rank's window at N = 4, minimum strip heights 8 / 4
set -euo pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_minry2
mkdir -p $OUT
for r in 8 4 8 4; do
  echo -n "minry=$r c1: "; LSQ_CG_RW_MINRY=$r timeout -k 10 200 python3 tools/cg_phase_probe.py c1 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (round(d[k]*1e3,1) if isinstance(d[k], float) else d[k]) for k in ('cg_normal','cg_data','cg_update','normal_kernel')})"
done
for c in c1 c3; do
  for r in 8 4 8 4; do
    LSQ_CG_RW_MINRY=$r timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/${c}_$r.json 2> $OUT/${c}_$r.err
    python3 -c "import json; d=json.load(open('$OUT/${c}_$r.json')); print('$c minry=$r', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'], d['config'].get('normal_kernel'))"
  done
done
for r in 8 4 8 4; do
  LSQ_CG_RW_MINRY=$r timeout -k 10 300 python3 bench.py --config c4y4 --dist --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4y4_$r.json 2> $OUT/c4y4_$r.err
  python3 -c "import json; d=json.load(open('$OUT/c4y4_$r.json')); print('c4y4 minry=$r', round(d['value']), d['solve_time_s'], d['solve_iters'])"
done
