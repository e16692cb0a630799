# round 4 (development): β fused into the block-Jacobi update — the whole -m gpu suite, smoke, then
# C4 with and without the fusion (LSQ_CG_FUSE_BETA 1 / 0, two runs each), C3
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4fb}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for i in 1 2; do
for fa in 1 0; do
  for cfg in c4 c3; do
    LSQ_CG_FUSE_BETA=$fa timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/${cfg}_fa${fa}_$i.json 2> $OUT/${cfg}_fa${fa}_$i.err || { echo "$cfg fa$fa failed"; tail -3 $OUT/${cfg}_fa${fa}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${cfg}_fa${fa}_$i.json')); print('$cfg fa$fa', round(d['value']), round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'BJ', d['solve_block_jacobi']['solve_iters'], round(d['solve_block_jacobi']['solve_time_s'],4))"
  done
done
done
