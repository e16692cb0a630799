# round 6: Aᵀu with the parts side by side (-DMF_AT_SPLIT=1) (lib_split.so) —
# the full GPU suite on it, then the LSQR A/B: base vs split (tools/r6/gpu_i.sh)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6k
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp tools/ab/lib_split.so lssurf_amd/liblsqsurf.so
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/k_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/k_tests.log; cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so; exit 1; }
tail -3 $OUT/k_tests.log
cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so
SKIP_PMC=1 bash tools/r6/gpu_i.sh r6k split
