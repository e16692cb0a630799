# round 4 (development): cProfile of smooth_fit end to end at C4 on the committed code
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4e2e}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/profile_e2e.py c4 3 > $OUT/e2e_c4_profile.txt 2>&1 || { echo "profile failed"; tail -5 $OUT/e2e_c4_profile.txt; exit 1; }
head -40 $OUT/e2e_c4_profile.txt | cut -c1-160
