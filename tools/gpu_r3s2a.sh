# GPU-box check at the start of round 3's second session: full GPU suite, smoke, the driver's
# default bench line, and rocprof kernel stats of the same bench command
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3s2a}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -3 $OUT/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
timeout -k 10 400 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
cat $OUT/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
echo ok > $OUT/ok
