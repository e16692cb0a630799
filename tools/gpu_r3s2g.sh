# multigrid set-up replayed as a graph: multigrid / distributed / smooth_fit GPU tests, then C4
# bench set-up times with the graph and eager (LSQ_MG_SETUP_EAGER)
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3s2g}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_dist.py tests/test_gpu_smooth_fit.py tests/test_gpu_dist_rccl.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in graph eager graph; do
  if [ $v = eager ]; then export LSQ_MG_SETUP_EAGER=1; else unset LSQ_MG_SETUP_EAGER; fi
  timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 50 --warmup 5 > $OUT/c4_$v.json 2> $OUT/c4_$v.err
  python3 -c "import json; d=json.load(open('$OUT/c4_$v.json')); print('$v', round(d['value']), 'MG', round(d['solve_time_s'],4), 'setup', round(d['solve_setup_s'],4), 'first', round(d['solve_setup_first_s'],4), d['solve_iters'])"
done
