# round 4, session q (closing check): the whole GPU suite, smoke(), the default bench line and the
# rocprofv3 kernel statistics of the bench command (graph packet batching off: DESIGN.md §3)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4q}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -20
[ $rc -le 1 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', round(d['value']), d['roofline']['frac'], d['roofline']['traffic'], round(d['solve_time_s'],4), d['solve_iters'], d['cpu_baseline']['value'])"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
python3 tools/mg_iter_trace.py $OUT/prof/run_kernel_trace.csv > $OUT/mg_iter_trace.txt && grep "iteration span" $OUT/mg_iter_trace.txt
