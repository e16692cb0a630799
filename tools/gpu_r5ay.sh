# round 5 late: same-box A/B at C5 and C4 — the closing library (70d8a45), the current one (update
# kernel at 5 waves per SIMD) and the current one capped at 4 waves per SIMD (LSQ_CG_BLOCK_WMAX=4)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ay}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp lssurf_amd/liblsqsurf.so tools/ab/lib_cur.so
for c in c5 c4; do
  for i in 1 2; do
    for v in r5closing cur w4; do
      cp tools/ab/lib_$v.so lssurf_amd/liblsqsurf.so
      timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-pmc --no-solve --steps 100 --warmup 10 > $OUT/${c}_${v}_$i.json 2> $OUT/${c}_${v}_$i.err || { echo "bench $c $v failed"; tail -3 $OUT/${c}_${v}_$i.err; cp tools/ab/lib_cur.so lssurf_amd/liblsqsurf.so; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${c}_${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c $v', round(d['value']), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()})"
    done
  done
done
cp tools/ab/lib_cur.so lssurf_amd/liblsqsurf.so
