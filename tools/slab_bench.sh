set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/slab
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for c in c4y8 c4y4; do
  timeout -k 10 300 python3 bench.py --config $c --dist --no-cpu --no-pmc --steps 400 --warmup 20 > $OUT/${c}_dist.json 2> $OUT/${c}_dist.err
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c4y8 --dist --steps 100 --warmup 10 --no-cpu --no-solve --no-pmc > $OUT/kt.json 2> $OUT/kt.err
echo ok > $OUT/ok
