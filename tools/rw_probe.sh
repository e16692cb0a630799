# wave-strip kernel probe (development): non-live role times (tools/cg_phase_probe.py) for the
# given library variant under several settings, then rocprof kernel stats of the default
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/rw_probe_$1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cp tools/ab/lib_$1.so lssurf_amd/liblsqsurf.so
for s in "X=1" "LSQ_CG_DBG=1" "LSQ_CG_RW_RY=8" "LSQ_CG_RW_RY=16" "LSQ_CG_RW_RY=24" "LSQ_CG_RW=0"; do
  env $s timeout -k 10 200 python3 tools/cg_phase_probe.py c4 2>/dev/null | tail -1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/cg_phase_probe.py c4 > $OUT/prof.log 2>&1
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')):
    if 'k_cg' in r['Name']: print(r['Name'][:50], r['Calls'], r['AverageNs'])
"
