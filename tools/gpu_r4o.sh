# round 4, session o (development): compute_E at C4 (tiled windows, 12.6 M columns) — smooth_fit
# with compute_E=True, one outer iteration; heartbeat every minute
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4o}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
( while true; do sleep 60; echo "heartbeat $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1100 python3 -u tools/compute_e_at.py c4 > $OUT/compute_e_c4.json 2> $OUT/compute_e_c4.err
rc=$?; echo "compute_E rc=$rc"; tail -3 $OUT/compute_e_c4.json; tail -3 $OUT/compute_e_c4.err
exit $rc
