# round 6: compute_E window geometry after the Schur split and batches — tile 16 / 24 nodes (margin 24)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6h}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for t in 16 24; do
  LSQ_E_TILE=$t timeout -k 10 400 python -u tools/compute_e_at.py c4 > $OUT/ce_c4_t$t.json 2>&1 || { echo "c4 t$t failed"; tail -20 $OUT/ce_c4_t$t.json; exit 1; }
  tail -1 $OUT/ce_c4_t$t.json | cut -c1-800
done
