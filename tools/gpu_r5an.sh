# round 5: C5 (2048²×12, 8 M points, one GPU) — one multigrid iteration's kernel trace and the bench
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5an}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --config c5 --no-cpu --no-pmc > $OUT/bench_c5.json 2> $OUT/prof.err || { echo "prof failed"; tail -3 $OUT/prof.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c5.json').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
python3 tools/mg_iter_trace.py $OUT/prof/run_kernel_trace.csv > $OUT/mg_iter_trace.txt && tail -30 $OUT/mg_iter_trace.txt
rm -f $OUT/prof/run_kernel_trace.csv
