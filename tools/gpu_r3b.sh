# round 3: C5 (anisotropic) on one GPU + C4 regression line
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3b}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 bench.py --config c5a --no-pmc --no-cpu --steps 100 --warmup 10 > $OUT/c5a.json 2> $OUT/c5a.err || echo "c5a rc=$?" >> $OUT/c5a.err
timeout -k 10 300 python3 bench.py --config c4 --no-pmc --no-cpu --steps 200 --warmup 20 > $OUT/c4.json 2> $OUT/c4.err || echo "c4 rc=$?" >> $OUT/c4.err
cat $OUT/c5a.json $OUT/c4.json
