# smooth_fit end to end at C4 (3 outer iterations) and the smooth_fit GPU tests, after the
# host-assembly and right-hand-side changes
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3s2f}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_smooth_fit.py tests/test_gpu_multi_device.py tests/test_gpu_aniso.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config c4 --e2e 3 > $OUT/e2e_$i.json 2> $OUT/e2e_$i.err
  python3 -c "import json; d=json.load(open('$OUT/e2e_$i.json')); print(d.get('wall_s'), {k: (round(v,3) if isinstance(v,float) else v) for k,v in d.get('timing',{}).items() if k!='lsq_last'})"
done
