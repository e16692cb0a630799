# round 6: k_xw_spmv's dispatch order (assembled LSQR, bench --op 1): XW_ORDER 1 (default: SELL rows first) vs 0
# (lib_xw0), one box, alternating; then the LSQR tests on the default build
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6p
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
  for lib in base xw0; do
    cp tools/ab/lib_$lib.so lssurf_amd/liblsqsurf.so
    timeout -k 10 300 python3 bench.py --op 1 --method lsqr --precond 1 --no-cpu --no-pmc --no-solve --steps 200 --warmup 20 > $OUT/c4op1_${lib}_$i.json 2> $OUT/c4op1_${lib}_$i.err || { echo "$lib failed"; tail -5 $OUT/c4op1_${lib}_$i.err; cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4op1_${lib}_$i.json').read().strip().splitlines()[-1]); print('pass $i $lib', round(d['value']), round(d['ms_per_step'],4))"
  done
done
cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsqr.py tests/test_gpu_aniso.py tests/test_gpu_edge_cases.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/p_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/p_tests.log; exit 1; }
tail -2 $OUT/p_tests.log
