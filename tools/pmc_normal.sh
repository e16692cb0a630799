# GPU-box PMC pass (development): SQ wait / activity counters of the CG kernels at C4
set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${1:-pmcn}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d $OUT/p1 -o run --output-format csv -- python3 $R/bench.py --config c4 --no-pmc --no-cpu --no-solve --steps 4 --warmup 2 > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY -d $OUT/p2 -o run --output-format csv -- python3 $R/bench.py --config c4 --no-pmc --no-cpu --no-solve --steps 4 --warmup 2 > $OUT/p2.log 2>&1
echo ok > $OUT/ok
