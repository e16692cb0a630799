# round 5: multigrid transfer kernels with 2 / 4 (default) / 8 columns per thread and trip (MG_RU,
# tools/build_variant.sh) — rocprofv3 kernel statistics of the c4 bench, the variant library swapped in
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5au}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp lssurf_amd/liblsqsurf.so tools/ab/lib_ru4.so
for i in 1 2; do
  for v in ru4 ru8 ru2; do
    cp tools/ab/lib_$v.so lssurf_amd/liblsqsurf.so
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${v}_$i -o run --output-format csv -- python3 bench.py --config c4 --no-cpu --no-pmc --steps 20 > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || { echo "$v failed"; tail -3 $OUT/${v}_$i.err; cp tools/ab/lib_ru4.so lssurf_amd/liblsqsurf.so; exit 1; }
    rm -f $OUT/${v}_$i/run_kernel_trace.csv
    python3 - $OUT/${v}_$i/run_kernel_stats.csv $OUT/${v}_$i.json $v <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = {r['Name'][r['Name'].find('k_'):][:18]: (int(r['Calls']), float(r['AverageNs']) / 1e3) for r in csv.DictReader(open(sys.argv[1]))}
print(sys.argv[3], 'MG', round(d['solve_time_s'], 4), {k: v for k, v in ks.items() if k.startswith(('k_mg_restrict(', 'k_mg_prolong(', 'k_mg_coarse'))})
PY
  done
done
cp tools/ab/lib_ru4.so lssurf_amd/liblsqsurf.so
