# round 5 (development): where the fused level-0 node gather + smoothing spends its time (kernel
# trace per phase switch; results wrong under LSQ_MG_ATQ_DBG)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5m}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for dbg in 0 1 2 3; do
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 LSQ_MG_ATQ_SMOOTH=1 LSQ_MG_ATQ_DBG=$dbg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$dbg -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 20 --warmup 5 > $OUT/prof$dbg.json 2> $OUT/prof$dbg.err || { echo "prof $dbg failed"; tail -3 $OUT/prof$dbg.err; exit 1; }
  grep -E "k_mg_atq_smooth|k_cg_dmf_atq|k_mg_smooth<12, false" $OUT/prof$dbg/run_kernel_stats.csv | cut -d, -f1-5
done
