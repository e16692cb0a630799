# GPU-box sweep (development): per-rank slab configs of C4 (c4y8 / c4y4, one rank's window at
# N = 8 / 4) under the strip-height and x-edge knobs, and full C4 as the regression check
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-sweep}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
run() {   # name, env..., -- bench args
    local name=$1; shift
    timeout -k 10 300 env "$@" > $OUT/$name.json 2> $OUT/$name.err
}
run c4y8_xe8 LSQ_CG_XE=8 python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --no-solve --steps 400 --warmup 20
run c4y8_xe1 LSQ_CG_XE=1 python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --no-solve --steps 400 --warmup 20
for ys in 4 12 16; do
  run c4y8_ys$ys LSQ_CG_YS=$ys python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --no-solve --steps 400 --warmup 20
done
run c4y4_xe8 LSQ_CG_XE=8 python3 bench.py --config c4y4 --dist --no-cpu --no-pmc --no-solve --steps 400 --warmup 20
run c4y4_xe1 LSQ_CG_XE=1 python3 bench.py --config c4y4 --dist --no-cpu --no-pmc --no-solve --steps 400 --warmup 20
run c4_xe8 LSQ_CG_XE=8 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20
echo ok > $OUT/ok
