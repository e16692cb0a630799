# round 4, session g (development): the tiled-window diag((AᵀA)⁻¹) against the full band factor at
# 256²×12 (786 k columns, band ≈ 97 tiles) per tile / margin, incl. the default 64 / 24
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4g}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
( while true; do sleep 60; echo "heartbeat $(date +%T)"; done ) & HB=$!
EWIN_COMBOS=16/16,32/16,32/24,64/24,64/32 timeout -k 10 900 python3 -u tools/ewin_probe.py t256 > $OUT/ewin_t256.jsonl 2> $OUT/ewin_t256.err
rc=$?; echo "ewin rc=$rc"; cat $OUT/ewin_t256.jsonl
kill $HB
exit $rc
