# round 5: the default bench and its rocprofv3 kernel statistics after the one-read factor change
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ah}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); r=d['roofline']; c=d['cpu_baseline']; print('default', round(d['value']), r['kernel'], round(r['frac'],3), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()}, 'traffic', r['traffic'], 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'cpu', round(c['value'],2), round(c.get('csr_port',{}).get('value',0),2))"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "prof failed"; tail -3 $OUT/prof.err; exit 1; }
python3 tools/mg_iter_trace.py $OUT/prof/run_kernel_trace.csv > $OUT/mg_iter_trace.txt && tail -22 $OUT/mg_iter_trace.txt
rm -f $OUT/prof/run_kernel_trace.csv
