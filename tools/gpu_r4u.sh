# round 4, session u (development): the driver's multi-process bench path at N = 2 with both RCCL ranks
# on the one GPU (--same-device: socket transport), a short run; the smooth_fit GPU tests and the C4 end-to-end time after the
# one-pass row weights; then the asymmetric level-0 V-cycle
# (LSQ_MG_DEG0_PRE: pre-smoothing degree below the post-smoothing degree) at C4 and C5a
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4u}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --same-device --steps 40 --warmup 10 > $OUT/bench_n2.json 2> $OUT/bench_n2.err
rc=$?; echo "rc=$rc"; tail -c 1500 $OUT/bench_n2.json; tail -5 $OUT/bench_n2.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_smooth_fit.py tests/test_gpu_multi_device.py -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --config c4 --e2e 3 > $OUT/e2e_c4.json 2> $OUT/e2e_c4.err || { echo "e2e failed"; tail -3 $OUT/e2e_c4.err; exit 1; }
cat $OUT/e2e_c4.json
timeout -k 10 300 python3 tools/profile_e2e.py c4 3 > $OUT/e2e_c4_profile.txt 2>&1 || { echo "profile failed"; exit 1; }
head -12 $OUT/e2e_c4_profile.txt
for cfg in c4 c5a; do
for v in "LSQ_MG_DEG0_PRE=2" "LSQ_MG_DEG0_PRE=1" "LSQ_MG_DEG0=3 LSQ_MG_DEG0_PRE=1" "LSQ_MG_DEG0=3 LSQ_MG_DEG0_PRE=2"; do
  tag=${cfg}_$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-pmc --steps 100 --warmup 10 > $OUT/$tag.json 2> $OUT/$tag.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$cfg $v', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'], round(d['solve_time_s']/max(d['solve_iters'],1)*1e3,3), 'ms/it')"
done
done
