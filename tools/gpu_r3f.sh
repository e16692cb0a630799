# round 3: C5 (anisotropic) full-size property test, bench line with PMC traffic, rocprof kernel stats
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3f}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_aniso.py -x -v --timeout 250 --timeout-method thread -k full_size > $OUT/test_full.log 2>&1 || { echo "full-size test failed"; tail -20 $OUT/test_full.log; exit 1; }
tail -2 $OUT/test_full.log
timeout -k 10 600 python3 bench.py --config c5a --cpu-iters 6 --steps 100 --warmup 10 > $OUT/c5a.json 2> $OUT/c5a.err || { echo "bench failed"; tail $OUT/c5a.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config c5a --steps 100 --warmup 10 --no-cpu --no-pmc \
    > $OUT/ktrace.json 2> $OUT/ktrace.err || { echo "rocprof failed"; tail $OUT/ktrace.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c5a.json'));print(d['value'],d['roofline']['frac'],d['roofline']['traffic'],d['cpu_baseline'],d['solve_time_s'],d['solve_iters'])"
