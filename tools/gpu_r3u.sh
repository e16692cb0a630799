set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3u}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_cgnr.py tests/test_gpu_aniso.py tests/test_gpu_dist.py tests/test_gpu_smooth_fit.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAIL|Error |error:|^E  |passed|failed" $OUT/tests.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/mg_trace.py c4 > $OUT/run.log 2>&1 || exit 1; cat $OUT/run.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/mg_trace.py c4 > $OUT/trace_run.log 2>&1; rc=$?; echo "trace rc=$rc"; tail -3 $OUT/trace_run.log
[ $rc -eq 0 ] || exit $rc
f=$(find $OUT/tr -name '*kernel_trace.csv' | head -1)
python3 $GRAFT_REPO_ROOT/tools/mg_trace.py analyse $f > $OUT/mg_iter.txt; tail -24 $OUT/mg_iter.txt
rm -rf $OUT/tr
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u bench.py --config c4 > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"; tail -c 1500 $OUT/bench.json
