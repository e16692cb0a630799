# round 5: wave strips walking alternate directions (halo rows read once) — normal-operator tests,
# the release_full_csr test, then the C4 bench A/B (LSQ_CG_RW_ALT 0 / 1 / 0 / 1) with PMC traffic
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5j}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_gpu_normal_rw.py tests/test_gpu_solve_sequence.py tests/test_gpu_cgnr.py tests/test_gpu_mg.py > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|^E  " $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for a in 0 1 0 1; do
  LSQ_CG_RW_ALT=$a timeout -k 10 400 python3 bench.py --no-cpu > $OUT/bench_alt$a.json 2> $OUT/bench_alt$a.err || { echo "bench alt=$a failed"; tail -5 $OUT/bench_alt$a.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_alt$a.json').read().strip().splitlines()[-1]); r=d['roofline']
print('alt=$a', round(d['value'],1), round(d['solve_time_s'],4), d['solve_iters'], {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()}, r['traffic_detail']['cg_normal'] if isinstance(r['traffic_detail'],dict) else None)"
done
