# round 6: A·v by rows (tools/ab/lib_rows.so, -DMF_FWD_ROWS=1) and the bf16 LSQR epilogue — the full GPU
# suite on it, then the LSQR A/B against the base build (tools/r6/gpu_i.sh)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6j
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp tools/ab/lib_rows.so lssurf_amd/liblsqsurf.so
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/j_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/j_tests.log; cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so; exit 1; }
tail -3 $OUT/j_tests.log
cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so
SKIP_PMC=1 bash tools/r6/gpu_i.sh r6j rows
# the LSQR epilogue's factor: lf_t copy (default) vs f64 (LSQ_BLOCK_EPI_LF=0), base build, alternating
for i in 1 2; do
  for lf in 1 0; do
    LSQ_BLOCK_EPI_LF=$lf timeout -k 10 300 python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/c4_lf${lf}_$i.json 2> $OUT/c4_lf${lf}_$i.err || { echo "lf$lf failed"; tail -5 $OUT/c4_lf${lf}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4_lf${lf}_$i.json').read().strip().splitlines()[-1]); print('pass $i lf$lf', round(d['value']), d['ms_per_step'], d['roofline']['frac'])"
  done
done
