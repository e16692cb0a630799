set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3s}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_errors_window.py tests/test_gpu_band.py tests/test_gpu_smooth_fit.py -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error |error:|^E  |passed|failed" $OUT/tests.log | head -40
timeout -k 10 500 python -u tools/ewin_probe.py t64 t128 > $OUT/probe.log 2>&1; echo "probe rc=$?"; grep name $OUT/probe.log
