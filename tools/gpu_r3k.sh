set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3k}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/mg_trace.py c4 > $OUT/trace_run.log 2>&1; rc=$?; echo "trace rc=$rc"; tail -3 $OUT/trace_run.log
[ $rc -eq 0 ] || exit $rc
f=$(find $OUT/tr -name '*kernel_trace.csv' | head -1)
python3 $GRAFT_REPO_ROOT/tools/mg_trace.py analyse $f > $OUT/mg_iter.txt; cat $OUT/mg_iter.txt | tail -30
rm -rf $OUT/tr
