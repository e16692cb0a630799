set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3m}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/mg_trace.py c4 > $OUT/trace_run.log 2>&1; rc=$?; echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find $OUT/tr -name '*kernel_trace.csv' | head -1)
python3 $GRAFT_REPO_ROOT/tools/mg_trace.py setup $f > $OUT/mg_setup.txt; cat $OUT/mg_setup.txt
gzip -c $f > $OUT/kernel_trace.csv.gz
rm -rf $OUT/tr
