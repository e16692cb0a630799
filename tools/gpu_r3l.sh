set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3l}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_aniso.py tests/test_gpu_dist.py -x -q --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for adb in 0 1; do
  LSQ_CG_ADB=$adb timeout -k 10 200 python -u tools/mg_trace.py c4 > $OUT/adb$adb.log 2>&1 || exit 1
  echo "adb=$adb $(tail -1 $OUT/adb$adb.log)"
done
for ch in 0.05,1.1 0.15,1.1 0.1,1.05 0.1,1.2 0.2,1.2 0.07,1.15; do
  LSQ_MG_CHEB=$ch timeout -k 10 200 python -u tools/mg_trace.py c4 > $OUT/ch$ch.log 2>&1 || exit 1
  echo "cheb=$ch $(tail -1 $OUT/ch$ch.log)"
done
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --no-cpu --no-pmc > $OUT/bench_c4.json 2> $OUT/bench_c4.log; echo "bench rc=$?"
python3 -c "
import json; d=json.load(open('$OUT/bench_c4.json')); print(round(d['value']), d['solve_iters'], round(d['solve_total_s'],4), d['roofline']['kernel_ms'])"
