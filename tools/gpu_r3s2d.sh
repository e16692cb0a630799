# Verification of the committed state: full GPU suite, smoke, driver-style bench line, rocprof
# kernel stats of the bench command, set-up trace, C5a bench
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3s2d}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print(d['value'], d['config']['normal_kernel'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['solve_time_s'], d['solve_setup_s'], d['solve_setup_first_s'], d['solve_iters'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
LSQ_SETUP_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --steps 20 --warmup 5 > $OUT/trace.json 2> $OUT/trace.err
grep "^setup" $OUT/trace.err | tail -24
timeout -k 10 400 python3 bench.py --config c5a --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/c5a.json 2> $OUT/c5a.err
python3 -c "import json; d=json.load(open('$OUT/c5a.json')); print('c5a', d['value'], d['config']['normal_kernel'], d['roofline']['kernel_ms'], d['solve_time_s'], d['solve_setup_s'], d['solve_iters'])"
echo ok > $OUT/ok
