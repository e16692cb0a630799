# Full GPU suite with the wave-strip normal operator as default, the multigrid set-up phases
# (LSQ_SETUP_TRACE), and the operator A/B (wave-strip vs ring) on C1 / C3 / c4y8 / C5a
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3s2c}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
LSQ_SETUP_TRACE=1 timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 20 --warmup 5 > $OUT/c4_trace.json 2> $OUT/c4_trace.err
grep "^setup" $OUT/c4_trace.err
for c in c1 c3 c5a; do
  for rw in 1 0; do
    LSQ_CG_RW=$rw timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-pmc --steps 100 --warmup 10 > $OUT/${c}_rw$rw.json 2> $OUT/${c}_rw$rw.err
    python3 -c "import json; d=json.load(open('$OUT/${c}_rw$rw.json')); print('$c rw=$rw', d['config'].get('normal_kernel'), round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'solve', round(d['solve_time_s'],4), d['solve_iters'])"
  done
done
for rw in 1 0; do
  LSQ_CG_RW=$rw timeout -k 10 300 python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4y8_rw$rw.json 2> $OUT/c4y8_rw$rw.err
  python3 -c "import json; d=json.load(open('$OUT/c4y8_rw$rw.json')); print('c4y8 rw=$rw', round(d['value']), 'solve', round(d['solve_time_s'],4), d['solve_iters'])"
done
echo ok > $OUT/ok
