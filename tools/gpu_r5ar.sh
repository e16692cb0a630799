# round 5: HBM bytes of the multigrid transfer kernels at C4 (k_mg_restrict / k_mg_prolong, level 0
# → 1 and back): rocprofv3 FETCH_SIZE and WRITE_SIZE in separate passes over a short multigrid solve
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ar}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -d $OUT/$c -o run --output-format csv -- python3 bench.py --config c4 --no-cpu --no-pmc --steps 5 --warmup 2 > $OUT/$c.json 2> $OUT/$c.err || { echo "pmc $c failed"; tail -3 $OUT/$c.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, collections, statistics, sys
out = sys.argv[1]
for c in ('FETCH_SIZE', 'WRITE_SIZE'):
    rows = list(csv.DictReader(open(f'{out}/{c}/run_counter_collection.csv')))
    agg = collections.defaultdict(list)
    for r in rows:
        n = r['Kernel_Name']
        if 'k_mg_restrict' in n or 'k_mg_prolong' in n or 'k_mg_smooth' in n or 'k_cg_normal_rw' in n:
            n = n[n.find('k_'):][:26]
            agg[(n, int(r['Grid_Size']))].append((float(r['Counter_Value']), int(r['End_Timestamp']) - int(r['Start_Timestamp'])))
    for (n, g), l in sorted(agg.items(), key=lambda kv: -kv[0][1])[:14]:
        v = statistics.median([a for a, b in l]); d = statistics.median([b for a, b in l])
        print(c, f'{n:28s} grid {g:9d} n={len(l):4d} {v/1e3:9.1f} MB  {d/1e3:7.1f} us')
PY
