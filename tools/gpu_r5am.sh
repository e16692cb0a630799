# round 5 late closing, part 2: the default bench (PMC traffic, CPU baselines), the rocprofv3 kernel
# statistics of the same command with one multigrid iteration's trace, compute_E and smooth_fit
# end to end at C4
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5am}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); r=d['roofline']; c=d['cpu_baseline']; print('default', round(d['value']), r['kernel'], round(r['frac'],3), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()}, 'traffic', r['traffic'], 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'cpu', round(c['value'],2), round(c.get('csr_port',{}).get('value',0),2))"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "prof failed"; tail -3 $OUT/prof.err; exit 1; }
python3 tools/mg_iter_trace.py $OUT/prof/run_kernel_trace.csv > $OUT/mg_iter_trace.txt && tail -22 $OUT/mg_iter_trace.txt
rm -f $OUT/prof/run_kernel_trace.csv
timeout -k 10 300 python3 bench.py --config c4 --e2e 3 > $OUT/e2e_c4.json 2> $OUT/e2e_c4.err || { echo "e2e failed"; tail -5 $OUT/e2e_c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/e2e_c4.json').read().strip().splitlines()[-1]); print('e2e', {k: d[k] for k in d if 'e2e' in k or 'iters' in k})" 2>/dev/null | cut -c1-400
timeout -k 10 600 python3 -u tools/compute_e_at.py c4 > $OUT/compute_e_c4.json 2> $OUT/compute_e_c4.err || { echo "compute_E failed"; tail -5 $OUT/compute_e_c4.err; exit 1; }
tail -1 $OUT/compute_e_c4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['timing']['E_window']; print('compute_E c4', round(d['wall_s'],1), round(e['time_s'],1), e['selfcheck_rel'], e['lanes'])"
