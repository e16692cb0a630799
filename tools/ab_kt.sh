# wave-strip class-compressed table A/B (development): forced-path parity, then non-live role times
# and bench lines with LSQ_CG_RW_KT = 1 (5 dim-2 class rows) and 0 (one row per t), alternating
set -euo pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_kt
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_normal_rw.py -x -q --timeout 280 --timeout-method thread 2>&1 | tail -2
for i in 1 2; do
  for kt in 1 0; do
    echo -n "kt=$kt: "; LSQ_CG_RW_KT=$kt timeout -k 10 200 python3 tools/cg_phase_probe.py c4 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(d[k]*1e3,1) for k in ('cg_normal','cg_data','cg_update')})"
  done
done
for kt in 1 0; do
  LSQ_CG_RW_KT=$kt timeout -k 10 300 python3 bench.py > $OUT/bench_kt$kt.json 2> $OUT/bench_kt$kt.err
  python3 -c "import json; d=json.loads(open('$OUT/bench_kt$kt.json').read().strip().splitlines()[-1]); print('kt=$kt', d['value'], d['roofline']['achieved'], d.get('solve_time_s'), d.get('config',{}).get('normal_kernel'))"
done
