# round 5 (development): GPU suite, default bench, C4 end to end (later solves' iterations with the
# carried ‖A‖ estimate), two RCCL ranks on the one card (the bench's multi-GPU self-check fields)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5b}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi_device.py tests/test_gpu_normal_rw.py tests/test_gpu_rz.py tests/test_gpu_smooth_fit.py tests/test_gpu_solve_sequence.py tests/test_gpu_tri.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
timeout -k 10 300 python3 bench.py --config c4 --e2e 3 > $OUT/e2e_c4.json 2> $OUT/e2e_c4.err || { echo "e2e failed"; tail -5 $OUT/e2e_c4.err; exit 1; }
cat $OUT/e2e_c4.json
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --same-device --config c4 --steps 100 --warmup 10 \
    > $OUT/c4_n2_same_device.json 2> $OUT/c4_n2_same_device.err || { echo "n2 failed"; tail -5 $OUT/c4_n2_same_device.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c4_n2_same_device.json'));print(d['ranks'], d['rank_iter_ms_device'])"
