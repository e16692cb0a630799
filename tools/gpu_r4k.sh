# round 4, session k (development): the fused data-row kernel — parity tests, the CGNR / multigrid
# tests, C4 bench fused vs the three-kernel path, and its kernel trace (time, registers, LDS)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4k}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_dfuse.py tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_atq_rw.py tests/test_gpu_dist.py tests/test_gpu_dist_rccl.py tests/test_gpu_smooth_fit.py -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -20
[ $rc -le 1 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for v in "LSQ_CG_DFUSE=1" "LSQ_CG_DFUSE=0" "LSQ_MG_ROWS=0"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_$tag.json 2> $OUT/c4_$tag.err || { tail -5 $OUT/c4_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4_$tag.json')); print('c4 $v', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'BJ', d['solve_block_jacobi']['solve_iters'], round(d['solve_block_jacobi']['solve_time_s'],4))"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
python3 tools/mg_iter_trace.py $OUT/prof/run_kernel_trace.csv > $OUT/mg_iter_trace.txt && tail -25 $OUT/mg_iter_trace.txt
