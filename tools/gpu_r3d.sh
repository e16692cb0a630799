# LSQR structured-operator kernel times at C4 (regression check)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --config c4 --method lsqr --precond 1 --no-solve --no-pmc --no-cpu --steps 200 --warmup 20 > $OUT/c4_lsqr1.json 2> $OUT/c4_lsqr1.err
timeout -k 10 300 python3 bench.py --config c4 --method lsqr --precond 3 --no-solve --no-pmc --no-cpu --steps 200 --warmup 20 > $OUT/c4_lsqr3.json 2> $OUT/c4_lsqr3.err
for f in c4_lsqr1 c4_lsqr3; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',d['value'],d['roofline']['kernel_ms'])"; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_aniso.py tests/test_gpu_lsqr.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; echo "tests rc=$?"; tail -2 $OUT/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_smooth_fit.py tests/test_gpu_band_precond.py -x -q --timeout 120 --timeout-method thread > $OUT/tests2.log 2>&1; echo "tests2 rc=$?"; tail -2 $OUT/tests2.log
