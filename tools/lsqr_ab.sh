# LSQR A/B on one GPU box: variants tools/ab/lib_<v>.so (tools/build_variant.sh) against tools/ab/lib_base.so,
# alternating on one box: LSQR + block-Jacobi it/s at C4, then a rocprofv3 kernel-trace of each
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-lsqr_ab}
shift || true
V="${*:-at6 fwd8}"
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0   # rocprofv3 and captured graph batches
for i in 1 2; do
  for lib in base $V; do
    cp tools/ab/lib_$lib.so lssurf_amd/liblsqsurf.so
    timeout -k 10 300 python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/c4_${lib}_$i.json 2> $OUT/c4_${lib}_$i.err || { echo "$lib failed"; tail -5 $OUT/c4_${lib}_$i.err; cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4_${lib}_$i.json').read().strip().splitlines()[-1]); print('pass $i $lib', round(d['value']), d['ms_per_step'])"
  done
done
for lib in base $V; do
  cp tools/ab/lib_$lib.so lssurf_amd/liblsqsurf.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$lib -o run --output-format csv -- python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 100 --warmup 10 > $OUT/prof_$lib.log 2>&1 || { echo "prof $lib failed"; tail -5 $OUT/prof_$lib.log; cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so; exit 1; }
  f=$(find $OUT/prof_$lib -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$lib" <<'EOF'
import csv, re, sys
for r in list(csv.reader(open(sys.argv[1])))[1:6]:
    m = re.search(r'k_\w+', r[0])
    print(sys.argv[2], m.group(0) if m else r[0][:30], r[1], round(float(r[3]) / 1e3, 1), 'us')
EOF
done
cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so
# SQ / TCC counters of the base build's LSQR kernels (separate passes, kernel-trace only)
[ -n "${SKIP_PMC:-}" ] && exit 0
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 20 --warmup 2 > $OUT/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -5 $OUT/pmc_sq.log; exit 1; }
python3 tools/pmc_summary.py $OUT/pmc_sq k_mf_ k_block_epi > $OUT/pmc_sq.txt && cat $OUT/pmc_sq.txt
timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 20 --warmup 2 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 20 --warmup 2 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -5 $OUT/pmc_write.log; exit 1; }
python3 tools/pmc_summary.py $OUT/pmc_fetch k_mf_ k_block_epi > $OUT/pmc_fetch.txt && python3 tools/pmc_summary.py $OUT/pmc_write k_mf_ k_block_epi > $OUT/pmc_write.txt && cat $OUT/pmc_fetch.txt $OUT/pmc_write.txt
