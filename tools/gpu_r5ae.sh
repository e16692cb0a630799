# round 5: k_cg_block with the next wave step's loads in flight during the block products;
# LSQ_CG_BLOCK_DBG=2 is the same binary without the prefetch (A/B)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ae}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_aniso.py tests/test_gpu_dist.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for dbg in 0 2; do
    LSQ_CG_BLOCK_DBG=$dbg timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/b${dbg}_$i.json 2> $OUT/b${dbg}_$i.err || { echo "bench failed"; tail -3 $OUT/b${dbg}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b${dbg}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('dbg=$dbg', round(d['value']), round(r['kernel_ms']['cg_update']*1e3,1), r['frac'])"
  done
done
