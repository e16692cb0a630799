# round 4, session e (development): the headline config against an independent solve (the CPU
# oracle's LSQR to the GPU solves' stopping rule at C4), then compute_E at C4
# (tiled windows) and smooth_fit end to end at C4 with its cProfile
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4e}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
( while true; do sleep 60; echo "heartbeat $(date +%T)"; done ) & HB=$!
timeout -k 10 900 python3 bench.py --config c4 --no-pmc --cpu-solve --steps 50 --warmup 10 > $OUT/c4_cpusolve.json 2> $OUT/c4_cpusolve.err
rc=$?; echo "cpu-solve rc=$rc"
[ $rc -eq 0 ] && python3 -c "import json; d=json.load(open('$OUT/c4_cpusolve.json')); c=d['cpu_baseline']; print('c4 cpu solve', c.get('solve_time_s'), c.get('solve_iters'), 'rel diff', c.get('solve_rel_diff_gpu_vs_cpu'), 'gpu', d['solve_time_s'], d['solve_iters'])"
kill $HB
