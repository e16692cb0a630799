# round 5 (development): where compute_E's band sweeps spend their time — kernel trace of the
# window path at 256²×12 (one lane), then PMC traffic of the sweep kernel alone
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5q}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LSQ_E_LANES=1 timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex k_band_sweep -d $OUT/pmc -o run --output-format csv -- python3 tools/compute_e_at.py t256 > $OUT/pmc.json 2> $OUT/pmc.err || { echo "pmc failed"; tail -3 $OUT/pmc.err; exit 1; }
python3 - "$OUT" <<'PY'
import csv, sys, glob
out = sys.argv[1]
f = glob.glob(f'{out}/pmc/*counter_collection.csv')
rows = list(csv.DictReader(open(f[0])))
tot = {}
n = 0
for r in rows:
    tot[r['Counter_Name']] = tot.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
print('sweep PMC totals', {k: round(v / 1e9, 2) for k, v in tot.items()}, 'GB-ish', len(rows), 'rows')
PY
