# wave-strip normal operator (k_cg_normal_rw): parity tests, then C4 bench A/B against the ring
# kernel (LSQ_CG_RW=0) on one box
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3s2b}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_cgnr.py tests/test_gpu_mg.py -x -v --timeout 120 --timeout-method thread > $OUT/cgnr_tests.log 2>&1 || { tail -30 $OUT/cgnr_tests.log; exit 1; }
tail -2 $OUT/cgnr_tests.log
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_rw.json 2> $OUT/c4_rw.err
LSQ_CG_RW=0 timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_ring.json 2> $OUT/c4_ring.err
python3 - <<'EOF' $OUT
import json, sys
for n in ('c4_rw', 'c4_ring'):
    d = json.load(open(f'{sys.argv[1]}/{n}.json'))
    print(n, d['config'].get('normal_kernel'), round(d['value']), 'it/s', d['roofline']['kernel_ms'], 'solve', round(d['solve_time_s'], 4), d['solve_iters'])
EOF
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 200 --warmup 20 > $OUT/c4_prof.json 2> $OUT/c4_prof.err
echo ok > $OUT/ok
