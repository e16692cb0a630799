# GPU-box A/B (development): ring depth (LSQ_CG_RING2) and strip height (LSQ_CG_YS) of the
# normal-stencil kernel on C4 and on one rank's window at N = 8 (c4y8)
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-sweep2}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
run() {   # name, env..., -- bench args
    local name=$1; shift
    timeout -k 10 300 env "$@" > $OUT/$name.json 2> $OUT/$name.err
}
B8="python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --no-solve --steps 400 --warmup 20"
B4="python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 200 --warmup 20"
for r in 0 1; do
  run c4_r${r} LSQ_CG_RING2=$r $B4
  run c4_r${r}_ys24 LSQ_CG_RING2=$r LSQ_CG_YS=24 $B4
  for ys in 8 12 16 20; do
    run c4y8_r${r}_ys$ys LSQ_CG_RING2=$r LSQ_CG_YS=$ys $B8
  done
done
run c4_r0_again LSQ_CG_RING2=0 $B4
echo ok > $OUT/ok
