# round 5 (development): compute_E at C4, window geometry × lanes sweep
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5h}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in "32 2" "32 4" "48 3"; do
  set -- $cfg
  LSQ_E_TILE=$1 LSQ_E_LANES=$2 timeout -k 10 400 python3 -u tools/compute_e_at.py c4 > $OUT/ce_t$1_l$2.json 2> $OUT/ce_t$1_l$2.err || { echo "compute_E $cfg failed"; tail -5 $OUT/ce_t$1_l$2.err; exit 1; }
  tail -1 $OUT/ce_t$1_l$2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['timing']['E_window']; print('t=$1 lanes=$2', round(d['wall_s'],1), round(e['time_s'],1), e['selfcheck_rel'], e['tile_products'])"
done
