# round 6: L2 hit rates of the LSQR kernels (one --pmc pass, kernel-trace only)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6s
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum -d $OUT/pmc_tcc -o run --output-format csv -- python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 20 --warmup 2 > $OUT/pmc_tcc.log 2>&1 || { echo "pmc tcc failed"; tail -5 $OUT/pmc_tcc.log; exit 1; }
python3 tools/pmc_summary.py $OUT/pmc_tcc k_mf_ k_block_epi > $OUT/pmc_tcc.txt && cat $OUT/pmc_tcc.txt
