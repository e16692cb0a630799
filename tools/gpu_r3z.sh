set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3z}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_cgnr.py tests/test_gpu_aniso.py tests/test_gpu_dist.py tests/test_gpu_smooth_fit.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAIL|Error |error:|^E  |passed|failed" $OUT/tests.log | head -30
[ $rc -eq 0 ] || exit $rc
for pm in 0 16384; do
  LSQ_MG_PERSIST=$pm timeout -k 10 200 python3 -u tools/mg_trace.py c4 > $OUT/run_p$pm.log 2>&1 || exit 1; echo "persist=$pm"; cat $OUT/run_p$pm.log
done
timeout -k 10 200 python3 -u tools/form_probe.py c4 > $OUT/form.log 2>&1 || exit 1; cat $OUT/form.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/mg_trace.py c4 > $OUT/trace_run.log 2>&1; rc=$?; echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find $OUT/tr -name '*kernel_trace.csv' | head -1)
python3 $GRAFT_REPO_ROOT/tools/mg_trace.py analyse $f > $OUT/mg_iter.txt; tail -26 $OUT/mg_iter.txt
rm -rf $OUT/tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tf -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/form_probe.py c4 > $OUT/trace_form.log 2>&1; rc=$?; echo "form trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find $OUT/tf -name '*kernel_stats.csv' | head -1); cp $f $OUT/form_kernel_stats.csv; head -16 $OUT/form_kernel_stats.csv | cut -d, -f1-5 | cut -c1-160
rm -rf $OUT/tf
