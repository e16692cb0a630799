# round 6, first GPU call: new tests, the full GPU suite, the default bench line
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6a}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_golden_depth.py tests/test_gpu_full_size.py -x -v --timeout 600 --timeout-method thread -m gpu > $OUT/new_tests.log 2>&1 || { echo "new tests failed"; tail -30 $OUT/new_tests.log; exit 1; }
tail -3 $OUT/new_tests.log
timeout -k 10 1500 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || { echo "suite failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['cpu_baseline'].get('host'), d.get('solve_time_s'), d.get('lsqr_iters_per_s'), d.get('solve_lsqr',{}).get('solve_roofline'))"
