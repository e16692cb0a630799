set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3x}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_cgnr.py tests/test_gpu_aniso.py tests/test_gpu_smooth_fit.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAIL|Error |error:|^E  |passed|failed" $OUT/tests.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config c4 > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"; python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','ms_per_step','solve_time_s','solve_iters')}); print(d.get('kernel_ms')); print(d.get('traffic_detail'))"
cd /tmp && export TMPDIR=/tmp
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_$set -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/cg_phase_probe.py c4 > $OUT/pmc_$set.log 2>&1 || exit 1
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT k_cg_ > $OUT/pmc.txt; cat $OUT/pmc.txt
rm -rf $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE
