set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3q}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --config c1 --steps 200 --warmup 20 --no-pmc --cpu-solve > $OUT/bench_c1_cpusolve.json 2> $OUT/bench_c1_cpusolve.log; echo "c1 rc=$?"
timeout -k 10 900 python -u bench.py --config c3 --steps 200 --warmup 20 --no-pmc --cpu-solve > $OUT/bench_c3_cpusolve.json 2> $OUT/bench_c3_cpusolve.log; echo "c3 rc=$?"
python3 - <<'P'
import json, os
out = os.environ['GRAFT_REPO_ROOT'] + '/gpurun_out/r3q'
for c in ('c1', 'c3'):
    try:
        d = json.load(open(f'{out}/bench_{c}_cpusolve.json'))
    except Exception as e:
        print(c, e); continue
    cb = d['cpu_baseline']
    print(c, 'gpu', d['solve_iters'], round(d['solve_total_s'], 4), 'cpu', cb.get('solve_iters'), cb.get('solve_time_s'), cb.get('solve_istop'), 'diff', cb.get('solve_rel_diff_gpu_vs_cpu'))
P
