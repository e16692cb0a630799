# round 4, session c (development): GPU suite on the lazy-formation + partitioned-coarse-level
# build, the C4 bench line, the rocprofv3 kernel trace of the bench with solves (graph packet
# capture off: DESIGN.md §5), C5a iteration counts of the round-3 commits, and the partitioned
# vs replicated coarse levels over 4 / 8 virtual ranks at C4
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4c}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_SEL:-} > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -20
[ $rc -le 1 ] || exit 1   # test failures: go on to the measurements; a crash or a time-out: stop
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --steps 200 --warmup 20 > $OUT/c4.json 2> $OUT/c4.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/c4.json')); print('c4', round(d['value']), 'frac', round(d['roofline']['frac'],3), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'setup', round(d['solve_setup_s'],4), 'form', round(d['device_formation_s'],3), 'bytes', d['config']['rank0_system']['device_bytes'])"
for v in "LSQ_CG_ATQ_RW=0" "LSQ_MG_PERSIST=4096 LSQ_MG_PWG=1" "LSQ_MG_PERSIST=16384 LSQ_MG_PWG=1"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_$tag.json 2> $OUT/c4_$tag.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/c4_$tag.json')); print('c4 $v', round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()}, 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
for n in 4 8; do
  for part in 1 0; do
    LSQ_MG_PART=$part timeout -k 10 300 python3 tools/vgroup_bench.py c4 $n > $OUT/vg_c4_${n}_p$part.json 2> $OUT/vg_c4_${n}_p$part.err || { echo "vgroup $n $part failed"; exit 1; }
    cat $OUT/vg_c4_${n}_p$part.json
  done
done
