# round 5: the block products' FMA chains split in two (even / odd i) in k_cg_block and the
# multigrid smoother — tests on the new build, then the A/B of the two builds (tools/ab_lib.sh)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5x}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_affine_blocks.py tests/test_gpu_dist.py tests/test_gpu_multi_device.py > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|^E  " $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 900 bash tools/ab_lib.sh old > $OUT/ab.log 2>&1 || { echo "ab failed"; tail -5 $OUT/ab.log; exit 1; }
for f in gpurun_out/ab_old/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$f'.split('/')[-1], round(d['value']), d.get('solve_time_s') and round(d['solve_time_s'],4), round(r['kernel_ms']['cg_update']*1e3,1))"; done
