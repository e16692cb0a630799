# round 5: is the normal / data kernels' slow-down after the faster update a clock effect?  For the
# closing library and the current one: rocprofv3 GRBM_GUI_ACTIVE per dispatch with the kernel trace
# (busy cycles ÷ duration = the clock the kernel ran at), c4 CG steps only
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ao}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp lssurf_amd/liblsqsurf.so tools/ab/lib_cur.so
for v in r5closing cur; do
  cp tools/ab/lib_$v.so lssurf_amd/liblsqsurf.so
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $OUT/$v -o run --output-format csv -- python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 40 --warmup 5 > $OUT/$v.json 2> $OUT/$v.err || { echo "pmc $v failed"; tail -3 $OUT/$v.err; cp tools/ab/lib_cur.so lssurf_amd/liblsqsurf.so; exit 1; }
done
cp tools/ab/lib_cur.so lssurf_amd/liblsqsurf.so
ls -R $OUT | head -20
