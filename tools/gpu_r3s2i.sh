# wave-strip gate (strips of < 8 rows when they fill a quarter of the slots): multigrid /
# distributed / wave-strip GPU tests, then C1 / C3 / C4 / one rank's window at N = 4, 8 lines
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3s2i}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_normal_rw.py tests/test_gpu_mg.py tests/test_gpu_dist.py tests/test_gpu_dist_rccl.py tests/test_gpu_cgnr.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in c1 c3 c4; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/$c.json 2> $OUT/$c.err
  python3 -c "import json; d=json.load(open('$OUT/$c.json')); print('$c', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'], d['config'].get('normal_kernel'))"
done
for c in c4y4 c4y8; do
  timeout -k 10 300 python3 bench.py --config $c --dist --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/$c.json 2> $OUT/$c.err
  python3 -c "import json; d=json.load(open('$OUT/$c.json')); print('$c', round(d['value']), d['solve_time_s'], d['solve_iters'], d['config'].get('normal_kernel'))"
done
