# round 5: same-box A/B of the closing library (70d8a45, tools/ab/lib_r5closing.so) against the
# current one (one read per factor entry), alternating, c4 CG steps only
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ai}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp lssurf_amd/liblsqsurf.so tools/ab/lib_cur.so
for i in 1 2 3; do
  for v in r5closing cur; do
    cp tools/ab/lib_$v.so lssurf_amd/liblsqsurf.so
    timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || { echo "bench $v failed"; tail -3 $OUT/${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()})"
  done
done
cp tools/ab/lib_cur.so lssurf_amd/liblsqsurf.so
