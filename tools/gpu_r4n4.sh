# round 4, closing (development): the driver's multi-process bench path on the committed code at
# N = 2 and N = 4 with every RCCL rank on the one GPU (--same-device: socket transport), short runs
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4n4}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --same-device --steps 40 --warmup 10 > $OUT/bench_n$n.json 2> $OUT/bench_n$n.err
  rc=$?; echo "n=$n rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/bench_n$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_n$n.json')); print('n=$n', round(d['value']), d['scaling'], 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'comm B/it', d.get('solve_comm_bytes_per_iter'), 'BJ', d['solve_block_jacobi']['solve_iters'], 'rel', d.get('solve_rel_diff_vs_block_jacobi'))"
done
