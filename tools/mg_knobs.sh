# multigrid coarsest-level size and power-step count (development): C4 bench solve lines
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-mg_knobs}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for kv in "9 10" "5 10" "3 10" "9 6" "5 6" "9 10"; do
  set -- $kv
  LSQ_MG_COARSE=$1 LSQ_MG_POW=$2 timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 20 --warmup 5 > $OUT/c$1_p$2.json 2> $OUT/c$1_p$2.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/c$1_p$2.json')); print('coarse $1 pow $2', 'MG', round(d['solve_time_s'],4), 'setup', round(d['solve_setup_s'],4), 'total', round(d['solve_total_s'],4), d['solve_iters'], 'dx', d['solve_rel_diff_vs_block_jacobi'])"
done
# the N > 1 bench path after this round's bench changes: two ranks sharing the one GPU
unset LSQ_MG_COARSE LSQ_MG_POW
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --same-device --config c4 --steps 20 --warmup 5 \
    > $OUT/c4_n2_same_device.json 2> $OUT/c4_n2_same_device.err
echo "n2 rc=$?"; tail -c 600 $OUT/c4_n2_same_device.json
