# One multigrid-PCG iteration of a rank's window (default c4y8, RCCL path at N = 1), kernel by kernel:
# rocprofv3 --kernel-trace of the bench with graph packets dispatched one by one, then tools/mg_iter_trace.py
set -uo pipefail
CFG=${1:-c4y8}
OUT=$GRAFT_REPO_ROOT/gpurun_out/rank_trace_$CFG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench.py --config $CFG --dist --no-cpu --no-pmc --steps 20 --warmup 5 > $OUT/b.log 2>&1 || { echo "prof failed"; tail -5 $OUT/b.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python3 tools/mg_iter_trace.py $f > $OUT/trace.txt && head -90 $OUT/trace.txt
