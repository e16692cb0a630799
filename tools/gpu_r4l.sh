# round 4, session l (development): PMC counters of the multigrid iteration's kernels at C4
# (LDS bank conflicts and waits of the coarse tile kernel, HBM bytes of the fused data rows,
# restriction and prolongation) — one rocprofv3 --pmc pass per counter set
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4l}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT"; do
  i=$((i+1))
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 180 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/mg_pmc_probe.py c4 6 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i done"
done
python3 $R/tools/pmc_summary.py $OUT k_mg_tile k_mg_restrict k_mg_prolong k_mg_smooth k_cg_dmf_fused k_cg_normal_rw k_cg_block k_mg_edge > $OUT/pmc_summary.txt
cat $OUT/pmc_summary.txt
