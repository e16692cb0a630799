# round 5 (development): the update kernel with its block products removed (LSQ_CG_BLOCK_DBG=1,
# results wrong) against the real one — is k_cg_block held by its memory pattern or its compute?
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5w}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
  for v in 0 1; do
    LSQ_CG_BLOCK_DBG=$v timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-solve --steps 300 --warmup 20 > $OUT/dbg${v}_$i.json 2> $OUT/dbg${v}_$i.err || { echo "dbg $v failed"; tail -3 $OUT/dbg${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/dbg${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('dbg=$v', round(d['value']), round(r['kernel_ms']['cg_update']*1e3,1), round(r['frac'],3), r['traffic_detail']['cg_update'])"
  done
done
