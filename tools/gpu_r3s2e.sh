# Evidence for the committed state: smoke, driver-style default bench line (PMC traffic passes),
# rocprof kernel stats of the bench command (--no-solve: see DESIGN §3 on the profiler crash),
# C5a and one rank's window at N = 8 (RCCL path at N = 1)
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3s2e}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
timeout -k 10 500 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); r=d['roofline']; print(round(d['value']), r['frac'], r['traffic'], r['kernel_ms'], d['solve_time_s'], d['solve_setup_s'], d['solve_iters'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --no-solve --steps 200 --warmup 20 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
timeout -k 10 400 python3 bench.py --config c5a --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/c5a.json 2> $OUT/c5a.err
python3 -c "import json; d=json.load(open('$OUT/c5a.json')); print('c5a', round(d['value']), d['config']['normal_kernel'], d['solve_time_s'], d['solve_setup_s'], d['solve_iters'])"
timeout -k 10 300 python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --steps 400 --warmup 20 > $OUT/c4y8.json 2> $OUT/c4y8.err
python3 -c "import json; d=json.load(open('$OUT/c4y8.json')); print('c4y8', round(d['value']), d['solve_time_s'], d['solve_iters'])"
echo ok > $OUT/ok
