# round 4, session x (development): the multigrid set-up with the coarse levels' power steps beside
# level 0's (LSQ_MG_POW_CONC 1, the default, vs 0) after the one-wave dense tile kernels: the MG /
# solve-sequence / smooth_fit GPU tests, then C4, C5a, C3 benches per variant
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4x}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_solve_sequence.py tests/test_gpu_smooth_fit.py -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
for cfg in c4 c5a c3; do
for v in "LSQ_MG_POW_CONC=1" "LSQ_MG_POW_CONC=0"; do
  tag=${cfg}_$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$cfg $v', 'setup', round(d['solve_setup_s']*1e3,2), 'ms solve', round(d['solve_time_s'],4), d['solve_iters'], 'first', round(d.get('solve_setup_first_s',0)*1e3,1))"
done
done
