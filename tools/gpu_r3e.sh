# round 3: aniso + dist GPU tests, LSQR structured-operator kernel times at C4
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3e}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_aniso.py tests/test_gpu_dist.py tests/test_gpu_smooth_fit.py -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1; echo "tests rc=$?"; tail -3 $OUT/tests.log
timeout -k 10 300 python3 bench.py --config c4 --method lsqr --precond 1 --no-solve --no-pmc --no-cpu --steps 200 --warmup 20 > $OUT/c4_lsqr1.json 2> $OUT/c4_lsqr1.err
python3 -c "import json;d=json.load(open('$OUT/c4_lsqr1.json'));print('lsqr1',d['value'],d['roofline']['kernel_ms'])"
