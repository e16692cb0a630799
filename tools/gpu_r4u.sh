# round 4, session u (development): the driver's multi-process bench path at N = 2 with both RCCL ranks
# on the one GPU (--same-device: socket transport), a short run
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4u}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --same-device --steps 40 --warmup 10 > $OUT/bench_n2.json 2> $OUT/bench_n2.err
rc=$?; echo "rc=$rc"; tail -c 1500 $OUT/bench_n2.json; tail -5 $OUT/bench_n2.err
exit $rc
