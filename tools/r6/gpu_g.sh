# round 6: the coarsest level by column count (LSQ_MG_COARSE_COLS, elongated lattices) — MG / dist
# tests, then the per-rank windows c4y8, c4y4, c5y8 (RCCL path at N = 1) and C4 with and without it
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6g}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_dist.py tests/test_gpu_dist_rccl.py tests/test_gpu_golden_depth.py tests/test_gpu_cgnr.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/g_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/g_tests.log; exit 1; }
tail -3 $OUT/g_tests.log
for i in 1 2; do
  for v in 1024 0; do
    for c in c4y8 c4y4 c5y8; do
      LSQ_MG_COARSE_COLS=$v timeout -k 10 300 python3 bench.py --config $c --dist --no-cpu --no-pmc --steps 100 --warmup 10 > $OUT/${c}_cc${v}_$i.json 2> $OUT/${c}_cc${v}_$i.err || { echo "$c $v failed"; tail -5 $OUT/${c}_cc${v}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${c}_cc${v}_$i.json').read().strip().splitlines()[-1]); print('$c cc$v', round(d['value']), d['solve_time_s'], d['solve_iters'], d['solve_setup_s'])"
    done
  done
done
LSQ_MG_COARSE_COLS=1024 timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 50 --warmup 10 > $OUT/c4_cc1024.json 2> $OUT/c4_cc1024.err || { echo "c4 failed"; tail -5 $OUT/c4_cc1024.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c4_cc1024.json').read().strip().splitlines()[-1]); print('c4 cc1024', round(d['value']), d['solve_time_s'], d['solve_iters'], d['solve_setup_s'])"
