# GPU-box A/B of one library under two environment settings (development), alternating:
#   bash tools/env_ab.sh TAG 'VAR=a' 'VAR=b' [configs…]   (default configs: c4 c4y8 c5y8)
# c4: the default bench (CGNR + block-Jacobi rate and the multigrid solve); cNyM: a rank's window
# through the RCCL path at N = 1 (its multigrid solve)
set -euo pipefail
TAG=$1; A=$2; B=$3; shift 3
CFGS=${*:-c4 c4y8 c5y8}
OUT=$GRAFT_REPO_ROOT/gpurun_out/envab_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for side in a b; do
    if [ $side = a ]; then E=$A; else E=$B; fi
    for c in $CFGS; do
      if [ $c = c4 ] || [ $c = c5 ]; then F=""; else F="--dist"; fi
      env $E timeout -k 10 300 python3 bench.py --config $c $F --no-cpu --no-pmc --steps 300 --warmup 20 \
        > $OUT/${c}_${side}_$i.json 2> $OUT/${c}_${side}_$i.err
    done
  done
done
echo ok > $OUT/ok
