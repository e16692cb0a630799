# Closing run (the round-6 one): the whole GPU suite and smoke() on the final tree, the default bench, the rocprofv3
# kernel-trace statistics of the bench command, and the torchrun path at N = 2 on the one card
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-closing}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); r=d['roofline']; print('default', round(d['value']), round(r['frac'],3), 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'lsqr', round(d['lsqr_iters_per_s']), 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof bench failed"; tail -5 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 2 --same-device --steps 100 --warmup 10 > $OUT/n2_same_device.json 2> $OUT/n2_same_device.err || { echo "n2 failed"; tail -5 $OUT/n2_same_device.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/n2_same_device.json').read().strip().splitlines()[-1]); print('n2', round(d['value']), 'MG', d.get('solve_time_s'), d.get('solve_iters'), d['rank_iter_ms_device'])"
