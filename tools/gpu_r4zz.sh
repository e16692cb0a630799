# round 4, closing profile: rocprofv3 kernel statistics and trace of the bench command on the
# committed code (graph packet batching off for the profiled run: DESIGN.md §3), one multigrid
# iteration extracted from the trace, then the bench itself (default: PMC passes, CPU baseline)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4zz}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/prof.json 2> $OUT/prof.err
rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/prof.err; exit 1; }
grep -E "k_cg_ad_xedge|k_cg_dmf_atq|k_cg_normal_rw|k_cg_block" $OUT/prof/run_kernel_stats.csv | cut -d, -f1-4
python3 tools/mg_iter_trace.py $OUT/prof/run_kernel_trace.csv > $OUT/mg_iter_trace.txt && tail -22 $OUT/mg_iter_trace.txt
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); r=d['roofline']; print('default', round(d['value']), r['kernel'], round(r['frac'],3), r['traffic'], r['algorithmic_bytes'], 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'setup', round(d['solve_setup_s']*1e3,2), 'form', round(d['device_formation_s'],3))"
