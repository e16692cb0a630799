# round 4, session f (development): compute_E at C4 (tiled windows) and smooth_fit end to end at C4
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4f}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --config c4 --e2e 3 > $OUT/e2e_c4.json 2> $OUT/e2e_c4.err; echo "e2e rc=$?"; cat $OUT/e2e_c4.json
timeout -k 10 300 python3 tools/profile_e2e.py c4 3 > $OUT/e2e_c4_profile.txt 2>&1; echo "profile rc=$?"; head -3 $OUT/e2e_c4_profile.txt
timeout -k 10 1000 python3 tools/compute_e_at.py c4 > $OUT/compute_e_c4.json 2> $OUT/compute_e_c4.err; echo "compute_E rc=$?"; tail -2 $OUT/compute_e_c4.json
