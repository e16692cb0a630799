# round 5: per-rank floors (one rank's window through the RCCL path at N = 1) and the other
# BASELINE configurations with the alternating wave strips — A/B LSQ_CG_RW_ALT on the slabs
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5n}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'], {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()})" $1 $2; }
for c in c4y8 c4y4 c5y8; do
  for a in 1 0; do
    LSQ_CG_RW_ALT=$a timeout -k 10 300 python3 bench.py --config $c --dist --no-cpu --no-pmc --steps 400 --warmup 20 > $OUT/${c}_alt$a.json 2> $OUT/${c}_alt$a.err || { echo "$c failed"; tail -3 $OUT/${c}_alt$a.err; exit 1; }
    summ $OUT/${c}_alt$a.json "$c alt=$a"
  done
done
for c in c1 c2 c3 c5; do
  timeout -k 10 400 python3 bench.py --config $c --no-cpu --no-pmc > $OUT/$c.json 2> $OUT/$c.err || { echo "$c failed"; tail -3 $OUT/$c.err; exit 1; }
  summ $OUT/$c.json "$c"
done
