# round 4, session w (development): the multigrid per-solve set-up (≤ 15 ms at C4) —
# the coarse levels' power steps beside level 0's (LSQ_MG_POW_CONC 1 default / 0),
# fewer power steps per level (LSQ_MG_POW) and one more level above a smaller dense coarsest
# (LSQ_MG_COARSE 5: ≤ 5 nodes per side instead of 9), at C4, C5a and C3, after the one-wave dense
# tile kernels' tests; the formation steps at C4
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4w}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lsqr.py tests/test_gpu_mg.py tests/test_gpu_smooth_fit.py tests/test_gpu_band.py tests/test_gpu_tri.py tests/test_gpu_solve_sequence.py -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
for cfg in c4 c5a c3; do
for v in "LSQ_MG_POW_CONC=1" "LSQ_MG_POW_CONC=0" "LSQ_MG_POW=7" "LSQ_MG_COARSE=5"; do
  tag=${cfg}_$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$cfg $v', 'setup', round(d['solve_setup_s']*1e3,2), 'ms solve', round(d['solve_time_s'],4), d['solve_iters'], 'first', round(d.get('solve_setup_first_s',0)*1e3,1))"
done
done
timeout -k 10 300 python3 tools/form_probe.py c4 2 > $OUT/form_probe_c4.jsonl 2> $OUT/form_probe_c4.err || { echo "form probe failed"; tail -3 $OUT/form_probe_c4.err; exit 1; }
cat $OUT/form_probe_c4.jsonl
