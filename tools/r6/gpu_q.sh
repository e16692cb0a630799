# round 6: the Aᵀu part gathers as buffer loads (LSQ_MF_AT_BUF=1, default) vs global loads (0), LSQR + block-Jacobi
# at C4, one box, alternating; then the LSQR tests and a kernel-trace of each
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6q
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsqr.py tests/test_gpu_aniso.py tests/test_gpu_full_size.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/q_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/q_tests.log; exit 1; }
tail -1 $OUT/q_tests.log
for i in 1 2; do
  for b in 1 0; do
    LSQ_MF_AT_BUF=$b timeout -k 10 300 python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/c4_buf${b}_$i.json 2> $OUT/c4_buf${b}_$i.err || { echo "buf$b failed"; tail -5 $OUT/c4_buf${b}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4_buf${b}_$i.json').read().strip().splitlines()[-1]); print('pass $i buf$b', round(d['value']), round(d['ms_per_step'],4))"
  done
done
for b in 1 0; do
  LSQ_MF_AT_BUF=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_buf$b -o run --output-format csv -- python3 bench.py --method lsqr --no-cpu --no-pmc --no-solve --steps 100 --warmup 10 > $OUT/prof_buf$b.log 2>&1 || { echo "prof failed"; exit 1; }
  f=$(find $OUT/prof_buf$b -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "buf$b" <<'PY'
import csv, re, sys
for r in list(csv.reader(open(sys.argv[1])))[1:5]:
    m = re.search(r'k_\w+', r[0])
    print(sys.argv[2], m.group(0) if m else r[0][:30], r[1], round(float(r[3]) / 1e3, 1), 'us')
PY
done
