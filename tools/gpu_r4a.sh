# round 4, session a (development): (1) C5a — does the untimed first solve change the timed
# solve's multigrid iteration count (61 -> 72 since the first-solve change)?  (2) the rocprofv3
# host crash of the bench with solves, with the process's library map for symbolising the stack.
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4a}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --config c5a --no-cpu --no-pmc --steps 50 --warmup 10 > $OUT/c5a.json 2> $OUT/c5a.err
rc=$?; echo "c5a rc=$rc"; [ $rc -eq 0 ] || exit 1
python3 -c "import json; d=json.load(open('$OUT/c5a.json')); print('c5a MG first', d['solve_iters_first'], 'timed', d['solve_iters'], 'dx', d['solve_rel_diff_first'], 'BJ', d['solve_block_jacobi']['solve_iters'])"
LSQ_BENCH_MAPS=$OUT/maps.txt timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
