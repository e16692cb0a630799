# GPU-box check (development): full GPU suite, then the per-rank slab benches (c4y8 / c4y4 over
# the RCCL path at N = 1), C4 on one GPU, and two RCCL ranks sharing the one GPU
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-check}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
for c in c4y8 c4y4; do
  timeout -k 10 300 python3 bench.py --config $c --dist --no-cpu --no-pmc --steps 400 --warmup 20 > $OUT/${c}_dist.json 2> $OUT/${c}_dist.err
done
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4.json 2> $OUT/c4.err
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --same-device --config c4 --steps 100 --warmup 10 \
    > $OUT/c4_n2_same_device.json 2> $OUT/c4_n2_same_device.err
echo ok > $OUT/ok
