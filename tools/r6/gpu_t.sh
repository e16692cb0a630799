# round 6: k_mf_spmtv's workgroup count (LSQ_MF_AT_WG: 2048 default, 1024, 512, 256) — its L2 hit rate is 43 %;
# fewer waves in flight shrink the per-XCD working set.  LSQR + block-Jacobi at C4, one box, alternating
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6t
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for i in 1 2; do
  for wg in 2048 1024 512 256; do
    LSQ_MF_AT_WG=$wg timeout -k 10 300 python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/c4_wg${wg}_$i.json 2> $OUT/c4_wg${wg}_$i.err || { echo "wg$wg failed"; tail -5 $OUT/c4_wg${wg}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4_wg${wg}_$i.json').read().strip().splitlines()[-1]); print('pass $i wg$wg', round(d['value']), round(d['ms_per_step'],4))"
  done
done
for wg in 2048 512; do
  LSQ_MF_AT_WG=$wg timeout -k 10 -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_wg$wg -o run --output-format csv -- python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 20 --warmup 2 > $OUT/pmc_wg$wg.log 2>&1 || { echo "pmc failed"; exit 1; }
  echo "wg$wg"; python3 tools/pmc_summary.py $OUT/pmc_wg$wg k_mf_spmtv
done
