# round 4, session m (development): one rank's share of C4 at N = 4 / 8 through the RCCL path at N = 1
# (the per-rank floors), then C4 against the CPU oracle's LSQR to the GPU solves' stopping rule
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4m}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "default bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', round(d['value']), d['roofline'], d['cpu_baseline'])"
for c in c4y4 c4y8; do
  timeout -k 10 300 python3 bench.py --config $c --dist --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/${c}_dist1.json 2> $OUT/${c}_dist1.err || { echo "$c failed"; tail -5 $OUT/${c}_dist1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${c}_dist1.json')); print('$c', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'BJ', d.get('solve_block_jacobi',{}).get('solve_iters'), round(d.get('solve_block_jacobi',{}).get('solve_time_s',0),4))"
done
( while true; do sleep 60; echo "heartbeat $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python3 bench.py --config c4 --no-pmc --cpu-solve --steps 50 --warmup 10 > $OUT/c4_cpusolve.json 2> $OUT/c4_cpusolve.err
rc=$?; echo "cpu-solve rc=$rc"
[ $rc -eq 0 ] && python3 -c "import json; d=json.load(open('$OUT/c4_cpusolve.json')); c=d['cpu_baseline']; print('c4 cpu solve', c.get('solve_time_s'), c.get('solve_iters'), 'rel diff', c.get('solve_rel_diff_gpu_vs_cpu'), 'gpu', d['solve_time_s'], d['solve_iters'])"
exit $rc
