R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_sq -o run --output-format csv -- python3 $R/bench.py --config c3 --no-pmc --no-cpu --no-solve --steps 4 --warmup 2 > $R/gpurun_out/pmc_sq.log 2>&1
