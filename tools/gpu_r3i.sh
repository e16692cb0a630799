set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3i}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_rccl.py -x -v --timeout 300 --timeout-method thread > $OUT/rccl.log 2>&1; rc=$?; echo "rccl rc=$rc"; tail -8 $OUT/rccl.log
[ $rc -eq 0 ] || exit $rc
for c in c4 c4y4 c4y8; do
timeout -k 10 300 python -u bench.py --dist --config $c --steps 200 --warmup 20 --no-cpu --no-pmc > $OUT/bench_${c}_dist.json 2> $OUT/bench_${c}_dist.log; rc=$?; echo "bench $c rc=$rc"
[ $rc -eq 0 ] || exit $rc
done
python - <<'P'
import json, os
out = os.environ['GRAFT_REPO_ROOT'] + '/gpurun_out/' + os.environ.get('R', 'r3i')
for c in ('c4', 'c4y4', 'c4y8'):
    d = json.load(open(f'{out}/bench_{c}_dist.json'))
    print(c, round(d['value']), 'it/s', d.get('solve_precond'), d.get('solve_iters'), 'its', round(d.get('solve_total_s', 0), 4), 's',
          'bj', d.get('solve_block_jacobi', {}).get('solve_iters'), round(d.get('solve_block_jacobi', {}).get('solve_total_s', 0), 4),
          'mg it/s', round(d.get('solve_iters_per_s') or 0))
P
