# round 6: the default build (bf16 LSQR epilogue, A·v at 8 waves per SIMD) through the full GPU suite,
# then the full-size module on the split Aᵀu build (lib_split.so), whose run in r6k failed in C2
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6l
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/l_tests.log 2>&1 || { echo "base tests failed"; tail -40 $OUT/l_tests.log; exit 1; }
tail -2 $OUT/l_tests.log
cp tools/ab/lib_split.so lssurf_amd/liblsqsurf.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/l_split.log 2>&1 || { echo "split full-size failed"; grep -E "PASSED|FAILED|^E " $OUT/l_split.log | head -20; cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so; exit 1; }
tail -2 $OUT/l_split.log
cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so
