# round 4 (development): the register-resident block factor kernel and the data-row CG start — the whole -m gpu suite, smoke,
# then C4 / C5a / C3 multigrid set-up and solve, and the default bench
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4bf}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for cfg in c4 c5a c3; do
  timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-pmc --steps 100 --warmup 10 > $OUT/$cfg.json 2> $OUT/$cfg.err || { echo "$cfg failed"; tail -3 $OUT/$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$cfg.json')); print('$cfg', round(d['value']), 'setup', round(d['solve_setup_s']*1e3,2), 'ms solve', round(d['solve_time_s'],4), d['solve_iters'], 'first', round(d.get('solve_setup_first_s',0)*1e3,1), 'BJ', d['solve_block_jacobi']['solve_iters'], 'rel', d.get('solve_rel_diff_vs_block_jacobi'))"
done
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); r=d['roofline']; print('default', round(d['value']), r['kernel'], round(r['frac'],3), 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'setup', round(d['solve_setup_s']*1e3,2), 'form', round(d['device_formation_s'],3), 'cpu', d['cpu_baseline']['value'])"
