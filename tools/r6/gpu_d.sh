# round 6: the multigrid tail kernel (k_mg_tail) — parity tests, then C4 and c4y8 (one rank's
# window at N = 8, RCCL path at N = 1) with and without it, alternating
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6d}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg_tail.py tests/test_gpu_mg.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/tail_tests.log 2>&1 || { echo "tail tests failed"; tail -40 $OUT/tail_tests.log; exit 1; }
tail -3 $OUT/tail_tests.log
for i in 1 2; do
  for v in on off; do
    if [ $v = off ]; then T=0; else T=4096; fi
    LSQ_MG_TAIL=$T timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 50 --warmup 10 > $OUT/c4_${v}_$i.json 2> $OUT/c4_${v}_$i.err || { echo "c4 $v failed"; tail -5 $OUT/c4_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4_${v}_$i.json').read().strip().splitlines()[-1]); print('c4 $v', round(d['value']), d['solve_time_s'], d['solve_iters'], d['solve_setup_s'])"
    LSQ_MG_TAIL=$T timeout -k 10 300 python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --steps 100 --warmup 10 > $OUT/c4y8_${v}_$i.json 2> $OUT/c4y8_${v}_$i.err || { echo "c4y8 $v failed"; tail -5 $OUT/c4y8_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4y8_${v}_$i.json').read().strip().splitlines()[-1]); print('c4y8 $v', round(d['value']), d['solve_time_s'], d['solve_iters'])"
  done
done
