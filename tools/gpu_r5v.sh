# round 5: the update kernel fills each node's removed dz column with zeros (whole-line stores,
# LSQ_CG_HOLE) — CGNR tests, then alternating C4 benches LSQ_CG_HOLE 1 / 0 with the NT variants
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5v}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_multi_device.py tests/test_gpu_solve_sequence.py > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|^E  " $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for v in "LSQ_CG_HOLE=1" "LSQ_CG_HOLE=0" "LSQ_CG_HOLE=1 LSQ_CG_NT=1" "LSQ_CG_HOLE=1 LSQ_CG_NT=7"; do
    tag=$(echo $v | tr ' =' '__')_$i
    env $v timeout -k 10 300 python3 bench.py --config c4 --no-cpu --steps 300 --warmup 20 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), round(r['kernel_ms']['cg_update']*1e3,1), round(r['frac'],3), r['traffic_detail']['cg_update'], 'MG', round(d['solve_time_s'],4))"
  done
done
