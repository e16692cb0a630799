# round 5: the wave-strip normal kernel's p / q stores non-temporal (LSQ_CG_RW_NT bits 1 / 2), c4
# CG steps, alternating on one box
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ap}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
  for nt in 0 1 2 3; do
    LSQ_CG_RW_NT=$nt timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/nt${nt}_$i.json 2> $OUT/nt${nt}_$i.err || { echo "bench failed"; tail -3 $OUT/nt${nt}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/nt${nt}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('nt=$nt', round(d['value']), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()})"
  done
done
