# round 5: the update kernel's non-temporal variants re-measured on the closing code (LSQ_CG_NT)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ab}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
  for nt in 5 1 0 4 7; do
    LSQ_CG_NT=$nt timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/nt${nt}_$i.json 2> $OUT/nt${nt}_$i.err || { echo "nt $nt failed"; tail -3 $OUT/nt${nt}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/nt${nt}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('NT=$nt', round(d['value']), round(r['kernel_ms']['cg_update']*1e3,1))"
  done
done
