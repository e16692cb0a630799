# isolate the rocprofv3 crash (development): current library with the previous bench.py; then
# the current bench with --no-solve
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-prof_check2}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp tools/bench_prev_dev.py bench_prev_dev.py
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof1 -o run --output-format csv -- python3 bench_prev_dev.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/prof1.json 2> $OUT/prof1.err
echo "prev bench under rocprof rc=$?"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof2 -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --no-solve --steps 200 --warmup 20 > $OUT/prof2.json 2> $OUT/prof2.err
echo "bench --no-solve under rocprof rc=$?"
