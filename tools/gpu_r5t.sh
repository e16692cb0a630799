# round 5: wave-strip heights with the alternating walk (halo rows now L2 hits) — LSQ_CG_RW_RY
# sweep on C4 and on one rank's window at N = 8 (c4y8, c5y8)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5t}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for ry in 0 16 13 10 0; do
  tag=c4_ry$ry
  env $( [ $ry -gt 0 ] && echo LSQ_CG_RW_RY=$ry ) timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'], round(d['roofline']['kernel_ms']['cg_normal']*1e3,1))"
done
for c in c4y8 c5y8; do
  for ry in 0 6 4 3 0; do
    tag=${c}_ry$ry
    env $( [ $ry -gt 0 ] && echo LSQ_CG_RW_RY=$ry ) timeout -k 10 300 python3 bench.py --config $c --dist --no-cpu --no-pmc --steps 300 --warmup 20 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'], round(d['roofline']['kernel_ms']['cg_normal']*1e3,1))"
  done
done
