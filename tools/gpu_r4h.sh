# round 4, session h (development): GPU suite (block-normal class tables, warm start over ranks),
# the C4 bench line, the row-streaming node gather at 2 / 4 rows per wave, and the C5a
# multigrid iteration counts of the round-3 commits (the 61 -> 72 question)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4h}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_SEL:-} > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -20
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --steps 200 --warmup 20 > $OUT/c4.json 2> $OUT/c4.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/c4.json')); print('c4', round(d['value']), 'frac', round(d['roofline']['frac'],3), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'setup', round(d['solve_setup_s'],4), 'form', round(d['device_formation_s'],3), 'bytes', d['config']['rank0_system']['device_bytes'])"
for v in "LSQ_CG_ATQ_RW=1 LSQ_CG_ATQ_RY=2" "LSQ_CG_ATQ_RW=1 LSQ_CG_ATQ_RY=4" "LSQ_BLK_TAB=0"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_$tag.json 2> $OUT/c4_$tag.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/c4_$tag.json')); print('c4 $v', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'form', round(d['device_formation_s'],3))"
done
bash tools/gpu_r4d.sh ${1:-r4h}
