# round 6: CGNR with the data rows' Ad·p forked beside the normal kernel (LSQ_CG_AD_FORK=1) — the CG
# tests (the new bit-identity test among them) and the LSQR tests on the default build (A·v dispatch
# order), then the C4 bench alternating the switch, and one LSQR bench
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6o
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_cgnr.py tests/test_gpu_lsqr.py tests/test_gpu_mg.py tests/test_gpu_full_size.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/o_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/o_tests.log; exit 1; }
tail -2 $OUT/o_tests.log
for i in 1 2; do
  for fk in 0 1; do
    LSQ_CG_AD_FORK=$fk timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --steps 400 --warmup 20 > $OUT/c4_fork${fk}_$i.json 2> $OUT/c4_fork${fk}_$i.err || { echo "fork$fk failed"; tail -5 $OUT/c4_fork${fk}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4_fork${fk}_$i.json').read().strip().splitlines()[-1]); print('pass $i fork$fk', round(d['value']), round(d['ms_per_step'],4), 'MG', d['solve_time_s'], d['solve_iters'], 'lsqr', round(d.get('lsqr_iters_per_s', 0)))"
  done
done
