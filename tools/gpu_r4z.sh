# round 4, session z (development): the whole -m gpu suite with the affine node blocks
# (lsq_set_column_blocks_affine) and smoke(); the default bench (formation after the runtime
# start) and the formation probe; the C4 end-to-end time
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4z}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR|^E  " $OUT/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', round(d['value']), d['roofline']['frac'], 'MG', round(d['solve_time_s'],4), d['solve_iters'], 'setup', round(d['solve_setup_s']*1e3,2), 'form', round(d['device_formation_s'],3), 'host', round(d['host_assembly_s'],3), 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 300 python3 tools/form_probe.py c4 2 > $OUT/form_probe_c4.jsonl 2> $OUT/form_probe_c4.err || { echo "form probe failed"; tail -3 $OUT/form_probe_c4.err; exit 1; }
tail -1 $OUT/form_probe_c4.jsonl
timeout -k 10 300 python3 bench.py --config c4 --e2e 3 > $OUT/e2e_c4.json 2> $OUT/e2e_c4.err || { echo "e2e failed"; tail -3 $OUT/e2e_c4.err; exit 1; }
cat $OUT/e2e_c4.json
