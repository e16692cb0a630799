set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3y}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u tools/form_probe.py c4 > $OUT/form.log 2>&1 || exit 1; cat $OUT/form.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/form_probe.py c4 > $OUT/trace_run.log 2>&1; rc=$?; echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find $OUT/tr -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats.csv; head -25 $OUT/kernel_stats.csv | cut -c1-200
f=$(find $OUT/tr -name '*memory_copy*stats*.csv' | head -1); [ -n "$f" ] && cp $f $OUT/copy_stats.csv
rm -rf $OUT/tr
