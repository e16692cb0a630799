# round 4, session r (development): one-rank RCCL groups replaying captured batches
# (LSQ_DIST_GRAPH=1) against the eager path — one rank's share of C4 at N = 8 / 4 through the RCCL
# path at N = 1, then the two-process RCCL tests with capture on
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4r}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in c4y8 c4y4; do
  for g in 0 1; do
    LSQ_DIST_GRAPH=$g timeout -k 10 300 python3 bench.py --config $c --dist --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/${c}_g$g.json 2> $OUT/${c}_g$g.err || { echo "$c g$g failed"; tail -5 $OUT/${c}_g$g.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${c}_g$g.json')); print('$c graph=$g', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'BJ', d.get('solve_block_jacobi',{}).get('solve_iters'), round(d.get('solve_block_jacobi',{}).get('solve_time_s',0),4), 'rel', d.get('solve_rel_diff_vs_block_jacobi'))"
  done
done
LSQ_DIST_GRAPH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_rccl.py -v --timeout 240 --timeout-method thread > $OUT/rccl_graph_tests.log 2>&1
rc=$?; tail -3 $OUT/rccl_graph_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/rccl_graph_tests.log | head -10
exit $rc
