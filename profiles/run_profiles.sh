#!/bin/bash
# GPU-box recipe for the committed profiles (run under gpurun from the repo root):
#   bench (N=1; it runs its own two rocprofv3 --pmc passes for roofline.traffic), bench over the
#   RCCL path (N=1), rocprofv3 kernel-trace stats of the bench, smooth_fit end to end (3 outer
#   iterations), and the 2-rank torchrun bench with both ranks on the one GPU (RCCL sockets).
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
TAG=${1:-r01}
CFG=${2:-c4}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 bench.py --config "$CFG" > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 python3 bench.py --config "$CFG" --dist --no-cpu --no-pmc > "$OUT/bench_dist1.json" 2> "$OUT/bench_dist1.err"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ktrace" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --config "$CFG" --steps 100 --warmup 10 --no-cpu --no-solve --no-pmc \
    > "$OUT/ktrace.json" 2> "$OUT/ktrace.err"
timeout -k 10 600 python3 bench.py --config "$CFG" --e2e 3 > "$OUT/e2e.json" 2> "$OUT/e2e.err"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --same-device --config "$CFG" --steps 100 --warmup 10 \
    > "$OUT/bench_n2_same_device.json" 2> "$OUT/bench_n2_same_device.err"
echo done > "$OUT/ok"
