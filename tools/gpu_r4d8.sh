# round 4 (development): where one rank's multigrid iteration goes at c4y8 (one rank's window of C4
# at N = 8, the per-rank floor of DESIGN §6): rocprofv3 kernel trace of the --dist bench at world 1
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4d8}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/prof.json 2> $OUT/prof.err
rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || { tail -5 $OUT/prof.err; exit 1; }
head -30 $OUT/prof/run_kernel_stats.csv | cut -d, -f1-5
