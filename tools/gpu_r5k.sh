# round 5: wave strips walking alternate directions + level-0 node gather fused with smoothing —
# tests, then C4 bench A/B (LSQ_CG_RW_ALT, LSQ_MG_ATQ_SMOOTH) with PMC traffic
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5k}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mg.py tests/test_gpu_normal_rw.py tests/test_gpu_solve_sequence.py tests/test_gpu_cgnr.py > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|^E  " $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for cfg in "1 1" "0 1" "1 0" "1 1" "0 0"; do
  set -- $cfg
  LSQ_CG_RW_ALT=$1 LSQ_MG_ATQ_SMOOTH=$2 timeout -k 10 400 python3 bench.py --no-cpu > $OUT/bench_a$1_f$2.json 2> $OUT/bench_a$1_f$2.err || { echo "bench $cfg failed"; tail -5 $OUT/bench_a$1_f$2.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_a$1_f$2.json').read().strip().splitlines()[-1]); r=d['roofline']
print('alt=$1 fuse=$2', round(d['value'],1), round(d['solve_time_s'],4), d['solve_iters'], {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()}, r['traffic_detail']['cg_normal'] if isinstance(r['traffic_detail'],dict) else None)"
done
