# round 5: the V-cycle's normal operator with two z rows in flight (k_cg_normal_rw<12, 2, false>) —
# parity tests, then alternating LSQ_CG_RW_PF2 = 1 / 0 on C4, C5 and c4y8 (multigrid solve times)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5p}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_normal_rw.py tests/test_gpu_mg.py tests/test_gpu_dist.py tests/test_gpu_smooth_fit.py > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|^E  " $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for pf in 1 0; do
    for c in c4 c5; do
      LSQ_CG_RW_PF2=$pf timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-pmc --steps 100 --warmup 10 > $OUT/${c}_pf${pf}_$i.json 2> $OUT/${c}_pf${pf}_$i.err || { echo "$c failed"; tail -3 $OUT/${c}_pf${pf}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${c}_pf${pf}_$i.json').read().strip().splitlines()[-1]); print('$c pf=$pf', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
    done
    LSQ_CG_RW_PF2=$pf timeout -k 10 300 python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --steps 200 --warmup 10 > $OUT/c4y8_pf${pf}_$i.json 2> $OUT/c4y8_pf${pf}_$i.err || { echo "c4y8 failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4y8_pf${pf}_$i.json').read().strip().splitlines()[-1]); print('c4y8 pf=$pf', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
  done
done
