# GPU-box A/B (development): the CG iteration's x-edge pass with 1 or 8 lanes per item on C4 / C3 / C1
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-xe}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for c in c4 c3 c1; do
  for xe in 1 8; do
    timeout -k 10 300 env LSQ_CG_XE=$xe python3 bench.py --config $c --no-cpu --no-pmc --steps 300 --warmup 20 > $OUT/${c}_xe$xe.json 2> $OUT/${c}_xe$xe.err
  done
done
echo ok > $OUT/ok
