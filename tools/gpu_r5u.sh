# round 5: minimum wave-strip height 3 (LSQ_CG_RW_RYMIN, was 4) — normal-operator tests, then
# A/B on the configurations the clamp reaches (c4y8, c4y4, C3) and C4 / c5y8 as controls
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5u}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_normal_rw.py tests/test_gpu_dist.py tests/test_gpu_cgnr.py > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|^E  " $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for m in 3 4 2; do
    for c in c4y8 c4y4 c3; do
      d=""; [ $c != c3 ] && d="--dist"
      LSQ_CG_RW_RYMIN=$m timeout -k 10 300 python3 bench.py --config $c $d --no-cpu --no-pmc --steps 300 --warmup 20 > $OUT/${c}_m${m}_$i.json 2> $OUT/${c}_m${m}_$i.err || { echo "$c failed"; tail -3 $OUT/${c}_m${m}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${c}_m${m}_$i.json').read().strip().splitlines()[-1]); print('$c min=$m', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'], round(d['roofline']['kernel_ms']['cg_normal']*1e3,1))"
    done
  done
done
