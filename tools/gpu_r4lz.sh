# round 4 (development): the whole -m gpu suite after the lazy interpolation weights, then the C4
# end-to-end time and its cProfile
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4lz}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --config c4 --e2e 3 > $OUT/e2e_c4.json 2> $OUT/e2e_c4.err || { echo "e2e failed"; tail -3 $OUT/e2e_c4.err; exit 1; }
cat $OUT/e2e_c4.json
timeout -k 10 300 python3 tools/profile_e2e.py c4 3 > $OUT/e2e_c4_profile.txt 2>&1 || { echo "profile failed"; exit 1; }
head -24 $OUT/e2e_c4_profile.txt | cut -c1-150
