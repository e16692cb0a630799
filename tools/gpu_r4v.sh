# round 4, session v (development): the whole -m gpu suite and smoke() on the committed code (one-pass
# row weights, parse_model column slices), the default bench (device_formation_s without host
# weights), then taller normal-operator strips (LSQ_CG_RW_RY 26 / 38: less halo, fewer waves) at C4
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4v}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -4 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', round(d['value']), d['roofline']['frac'], 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'form', round(d['device_formation_s'],3), 'host', round(d['host_assembly_s'],3))"
for v in "LSQ_CG_RW_RY=26" "LSQ_CG_RW_RY=38"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_$tag.json 2> $OUT/c4_$tag.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/c4_$tag.json')); print('c4 $v', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
done
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4.json 2> $OUT/c4.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/c4.json')); print('c4', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
