# round 4, session s (development): Ad·p with two points per trip — CGNR tests, C4 bench, kernel stats
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4s}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_cgnr.py tests/test_gpu_atq_rw.py tests/test_gpu_mg.py -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -20
[ $rc -le 1 ] || exit 1
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_$i.json 2> $OUT/c4_$i.err || { tail -5 $OUT/c4_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4_$i.json')); print('c4', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
grep -E "k_cg_ad_xedge|k_cg_dmf_atq|k_cg_normal_rw|k_cg_block" $OUT/prof/run_kernel_stats.csv | cut -d, -f1-4
