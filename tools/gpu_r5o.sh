# round 5: wave-strip shifts as DPP wave_shl/wave_shr instead of ds_bpermute — parity tests, then
# the A/B of the two builds (tools/ab_lib.sh: C4 bench + multigrid solve, c4y8)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5o}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_normal_rw.py tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_dist.py > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|^E  " $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 900 bash tools/ab_lib.sh bperm > $OUT/ab.log 2>&1 || { echo "ab failed"; tail -5 $OUT/ab.log; exit 1; }
for f in gpurun_out/ab_bperm/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$f'.split('/')[-1], round(d['value']), d.get('solve_time_s') and round(d['solve_time_s'],4), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()})"; done
