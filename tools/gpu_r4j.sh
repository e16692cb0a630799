# round 4, session j (development): C5a on round 3's early point cloud (seed id 10) with the
# current build; smooth_fit end to end at C4 with its cProfile; the tiled-window σ against the full
# band at 256²×12
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4j}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
( while true; do sleep 60; echo "heartbeat $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python3 -u tools/c5a_conv.py c5a 10 > $OUT/c5a_conv_seed10.jsonl 2> $OUT/c5a_conv_seed10.err || { echo "conv failed"; tail -3 $OUT/c5a_conv_seed10.err; exit 1; }
head -4 $OUT/c5a_conv_seed10.jsonl
timeout -k 10 300 python3 bench.py --config c4 --e2e 3 > $OUT/e2e_c4.json 2> $OUT/e2e_c4.err || { echo "e2e failed"; tail -3 $OUT/e2e_c4.err; exit 1; }
cat $OUT/e2e_c4.json
timeout -k 10 300 python3 tools/profile_e2e.py c4 3 > $OUT/e2e_c4_profile.txt 2>&1 || { echo "profile failed"; exit 1; }
head -30 $OUT/e2e_c4_profile.txt
EWIN_COMBOS=16/16,32/16,32/24,64/24,64/32 timeout -k 10 700 python3 -u tools/ewin_probe.py t256 > $OUT/ewin_t256.jsonl 2> $OUT/ewin_t256.err
rc=$?; echo "ewin rc=$rc"; cat $OUT/ewin_t256.jsonl; tail -3 $OUT/ewin_t256.err
exit $rc
