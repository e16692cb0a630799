# round 5: LSQR block-Jacobi epilogue on affine blocks (k_block_epi_aff) — the LSQR / CGNR GPU
# tests, then the c4 LSQR bench with and without it (LSQ_BLOCK_EPI_AFF=0: k_block_epi), alternating
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5aj}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lsqr.py tests/test_gpu_cgnr.py tests/test_gpu_full_size.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for a in 1 0; do
    LSQ_BLOCK_EPI_AFF=$a timeout -k 10 300 python3 bench.py --config c4 --method lsqr --no-cpu --no-pmc --no-solve --steps 100 --warmup 10 > $OUT/aff${a}_$i.json 2> $OUT/aff${a}_$i.err || { echo "bench failed"; tail -3 $OUT/aff${a}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/aff${a}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('aff=$a', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()})"
  done
done
