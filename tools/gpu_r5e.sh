# round 5 (development): the whole GPU suite (x every 4th CG step, interior-only window sweeps),
# the default bench, then compute_E at C4 (round 4: 477 s)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5e}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); r=d['roofline']; c=d['cpu_baseline']; print('default', round(d['value']), r['kernel'], round(r['frac'],3), r['kernel_ms'], 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'cpu', c['value'], c.get('csr_port',{}).get('value'))"
timeout -k 10 900 python3 -u tools/compute_e_at.py c4 > $OUT/compute_e_c4.json 2> $OUT/compute_e_c4.err || { echo "compute_E failed"; tail -5 $OUT/compute_e_c4.err; exit 1; }
tail -1 $OUT/compute_e_c4.json
