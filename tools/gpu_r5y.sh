# round 5: one rank's multigrid iteration at N = 8 (c4y8 through the RCCL path at N = 1), traced
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5y}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/prof.json 2> $OUT/prof.err || { echo "prof failed"; tail -3 $OUT/prof.err; exit 1; }
python3 tools/mg_iter_trace.py $OUT/prof/run_kernel_trace.csv > $OUT/mg_iter_trace.txt && cat $OUT/mg_iter_trace.txt | tail -40
rm -f $OUT/prof/run_kernel_trace.csv
