# round 6: same-box A/B of the update kernel's factor-read form (LSQ_CG_BLOCK_RC 1 = one read per entry,
# 0 = row and column apart) at C5 and C4, two alternating passes
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6b}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in c5 c4; do
  for i in 1 2; do
    for v in 1 0; do
      LSQ_CG_BLOCK_RC=$v timeout -k 10 400 python3 bench.py --config $c --no-cpu --no-pmc --no-solve --steps 100 --warmup 10 > $OUT/${c}_rc${v}_$i.json 2> $OUT/${c}_rc${v}_$i.err || { echo "bench $c $v failed"; tail -3 $OUT/${c}_rc${v}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${c}_rc${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c rc$v', round(d['value']), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()})"
    done
  done
done
