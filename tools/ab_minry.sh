# wave-strip gate A/B (development): the ring kernel below LSQ_CG_RW_MINRY rows per strip (default
# 8).  Non-live role times at C3 and the C4 multigrid solve (its level 1 has 4-row strips) and the
# N = 8 window, for minimum strip heights 8 / 4
set -euo pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_minry
mkdir -p $OUT
for r in 8 4 8 4; do
  echo -n "minry=$r c3: "; LSQ_CG_RW_MINRY=$r timeout -k 10 200 python3 tools/cg_phase_probe.py c3 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (round(d[k]*1e3,1) if isinstance(d[k], float) else d[k]) for k in ('cg_normal','cg_data','cg_update','normal_kernel')})"
done
for r in 8 4 8 4; do
  LSQ_CG_RW_MINRY=$r timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/c4_$r.json 2> $OUT/c4_$r.err
  python3 -c "import json; d=json.load(open('$OUT/c4_$r.json')); print('c4 minry=$r', round(d['value']), 'MG', round(d['solve_time_s'],4), 'setup', round(d['solve_setup_s'],4), d['solve_iters'])"
done
for r in 8 4; do
  LSQ_CG_RW_MINRY=$r timeout -k 10 300 python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --steps 400 --warmup 20 > $OUT/c4y8_$r.json 2> $OUT/c4y8_$r.err
  python3 -c "import json; d=json.load(open('$OUT/c4y8_$r.json')); print('c4y8 minry=$r', round(d['value']), d['solve_time_s'], d['solve_iters'])"
done
