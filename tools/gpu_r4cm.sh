# round 4 (development): wave strips numbered down the rows first (LSQ_CG_RW_CM=1: vertical
# neighbours, which share halo rows, adjacent in an XCD's chunk) against row-major (0) — the
# normal operator's tests under CM=1, then C4 with PMC traffic (two runs each), C5a, c4y8 rank
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4cm}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LSQ_CG_RW_CM=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_normal_rw.py tests/test_gpu_cgnr.py tests/test_gpu_mg.py -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
for cm in 0 1; do
  LSQ_CG_RW_CM=$cm timeout -k 10 300 python3 bench.py --config c4 --no-cpu --steps 200 --warmup 20 > $OUT/c4_cm${cm}_$i.json 2> $OUT/c4_cm${cm}_$i.err || { echo "c4 cm$cm failed"; tail -3 $OUT/c4_cm${cm}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4_cm${cm}_$i.json')); r=d['roofline']; t=r['traffic_detail']; print('c4 cm$cm', round(d['value']), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()}, 'normal traffic', round(t['cg_normal']['total']/1e9,3) if isinstance(t, dict) else t, 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
done
done
for cm in 0 1; do
  LSQ_CG_RW_CM=$cm timeout -k 10 300 python3 bench.py --config c5a --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/c5a_cm$cm.json 2> $OUT/c5a_cm$cm.err || { echo "c5a cm$cm failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5a_cm$cm.json')); print('c5a cm$cm', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
  LSQ_CG_RW_CM=$cm timeout -k 10 300 python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --steps 100 --warmup 10 > $OUT/c4y8_cm$cm.json 2> $OUT/c4y8_cm$cm.err || { echo "c4y8 cm$cm failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4y8_cm$cm.json')); print('c4y8 cm$cm', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
done
