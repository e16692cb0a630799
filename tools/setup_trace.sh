# per-solve set-up phases of the C4 multigrid solve (LSQ_SETUP_TRACE), development
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-setup_trace}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
LSQ_SETUP_TRACE=1 timeout -k 10 300 python3 bench.py --config ${2:-c4} --no-cpu --no-pmc --steps 20 --warmup 5 > $OUT/trace.json 2> $OUT/trace.err
grep "^setup" $OUT/trace.err
