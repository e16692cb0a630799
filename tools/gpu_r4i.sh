# round 4, session i (development): the C5a convergence curve of the current build and of the
# builds before / after 708e2d2 (the 61 -> 72 multigrid iteration change), then the wave-strip
# normal operator at shorter strips (more waves per SIMD: LSQ_CG_RW_RY) and the fused small-level
# restriction at C4
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4i}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_multi_device.py tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python3 -u tools/c5a_conv.py c5a > $OUT/c5a_conv_head.jsonl 2> $OUT/c5a_conv_head.err || { echo "conv head failed"; tail -3 $OUT/c5a_conv_head.err; exit 1; }
cat $OUT/c5a_conv_head.jsonl
for c in 5ce97ea 708e2d2; do
  cp tools/c5a_conv.py tools/ab/bisect/$c/tools/ 2>/dev/null || { mkdir -p tools/ab/bisect/$c/tools && cp tools/c5a_conv.py tools/ab/bisect/$c/tools/; }
  (cd tools/ab/bisect/$c && timeout -k 10 300 python3 -u tools/c5a_conv.py c5a > $OUT/c5a_conv_$c.jsonl 2> $OUT/c5a_conv_$c.err) || { echo "conv $c failed"; tail -3 $OUT/c5a_conv_$c.err; exit 1; }
  echo "== $c"; cat $OUT/c5a_conv_$c.jsonl
done
for v in "LSQ_CG_RW_RY=13" "LSQ_CG_RW_RY=10" "LSQ_MG_RES_FUSE=0"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_$tag.json 2> $OUT/c4_$tag.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/c4_$tag.json')); print('c4 $v', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
done
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4.json 2> $OUT/c4.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/c4.json')); print('c4', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'form', round(d['device_formation_s'],3))"
