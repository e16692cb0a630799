# round 5 late: same-box A/B at C5 of the closing library (70d8a45) against the current one, CG steps
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ax}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp lssurf_amd/liblsqsurf.so tools/ab/lib_cur.so
for i in 1 2; do
  for v in r5closing cur; do
    cp tools/ab/lib_$v.so lssurf_amd/liblsqsurf.so
    timeout -k 10 300 python3 bench.py --config c5 --no-cpu --no-pmc --no-solve --steps 100 --warmup 10 > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || { echo "bench $v failed"; tail -3 $OUT/${v}_$i.err; cp tools/ab/lib_cur.so lssurf_amd/liblsqsurf.so; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()})"
  done
done
cp tools/ab/lib_cur.so lssurf_amd/liblsqsurf.so
