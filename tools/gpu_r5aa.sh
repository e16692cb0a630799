# round 5: ranks replay their replicated coarse levels' V-cycle from a captured hipGraph
# (LSQ_MG_RGRAPH) — distributed tests, then A/B on one rank's windows and C4 through the RCCL path
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5aa}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_dist_rccl.py tests/test_gpu_multi_device.py tests/test_gpu_mg.py > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|^E  " $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for g in 1 0; do
    for c in c4y8 c4y4 c5y8 c4; do
      LSQ_MG_RGRAPH=$g timeout -k 10 300 python3 bench.py --config $c --dist --no-cpu --no-pmc --steps 100 --warmup 10 > $OUT/${c}_g${g}_$i.json 2> $OUT/${c}_g${g}_$i.err || { echo "$c failed"; tail -3 $OUT/${c}_g${g}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${c}_g${g}_$i.json').read().strip().splitlines()[-1]); print('$c rgraph=$g', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
    done
  done
done
