# round 5 (development): the class-compressed coarse tile kernel — multigrid tests, same-box A/B of
# LSQ_MG_TILE_KT = 0 (k_mg_tile) / 1 (scalar coefficients) / 2 (LDS coefficients) on the C4 bench's
# multigrid solve, and a kernel trace of one multigrid iteration with the default
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5c}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
for kt in 0 2 1 2 0; do
  LSQ_MG_TILE_KT=$kt timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --steps 100 --warmup 10 > $OUT/bench_kt$kt.json 2> $OUT/bench_kt$kt.err || { echo "bench kt=$kt failed"; tail -5 $OUT/bench_kt$kt.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_kt$kt.json')); print('kt=$kt', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'rel', d['solve_rel_diff_vs_block_jacobi'])"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 50 --warmup 10 > $OUT/prof.json 2> $OUT/prof.err
rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/prof.err; exit 1; }
python3 tools/mg_iter_trace.py $OUT/prof/run_kernel_trace.csv > $OUT/mg_iter_trace.txt && tail -22 $OUT/mg_iter_trace.txt
