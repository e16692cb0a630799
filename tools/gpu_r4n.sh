# round 4, session n (development): the four-lanes-per-node gather — parity tests, C4 A/B against the
# one-lane kernel, and a kernel trace of the bench (multigrid iteration breakdown)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4n}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_atq_rw.py tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -20
[ $rc -le 1 ] || exit 1
for v in "LSQ_CG_ATQ_RW=0" "LSQ_CG_ATQ_RW=4" "LSQ_CG_ATQ_RW=0" "LSQ_CG_ATQ_RW=4"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_$tag.json 2> $OUT/c4_$tag.err || { tail -5 $OUT/c4_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4_$tag.json')); print('c4 $v', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'BJ', d['solve_block_jacobi']['solve_iters'], round(d['solve_block_jacobi']['solve_time_s'],4))"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
python3 tools/mg_iter_trace.py $OUT/prof/run_kernel_trace.csv > $OUT/mg_iter_trace.txt && tail -22 $OUT/mg_iter_trace.txt
