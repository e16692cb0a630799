# bf16 vs fp32 node-block factors (development): GPU suite on the default (bf16) build, then C4
# bench lines of both builds, alternating
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab_lf}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
cp lssurf_amd/liblsqsurf.so /tmp/keep.so
for i in 1 2; do
  for lib in bf16 f32; do
    cp tools/ab/lib_$lib.so lssurf_amd/liblsqsurf.so
    timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_${lib}_$i.json 2> $OUT/c4_${lib}_$i.err
    python3 -c "import json; d=json.load(open('$OUT/c4_${lib}_$i.json')); print('$lib', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'frac', round(d['roofline']['frac'],3), 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'BJ', round(d['solve_block_jacobi']['solve_time_s'],4), d['solve_block_jacobi']['solve_iters'], 'LSQR', d['solve_lsqr']['solve_iters'], 'dx', d['solve_rel_diff_vs_lsqr'])"
  done
done
cp /tmp/keep.so lssurf_amd/liblsqsurf.so
echo ok > $OUT/ok
