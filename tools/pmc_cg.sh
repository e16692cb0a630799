#!/bin/bash
# PMC passes over the CGNR probe (tools/cg_phase_probe.py): one rocprofv3 run per counter set,
# output under gpurun_out/$1.  Usage (GPU box): bash tools/pmc_cg.sh <outdir> [config]
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$1; CFG=${2:-c4}
mkdir -p $OUT && cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/cg_phase_probe.py $CFG > $OUT/p$i.log 2>&1 || exit 1
done
