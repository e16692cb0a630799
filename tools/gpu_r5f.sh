# round 5 (development): compute_E at C4 with the timing breakdown, default windows (64 / 24) and
# 32-node tiles; the per-rank window of C5 at N = 8 (c5y8) through the RCCL path at N = 1
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5f}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --config c5y8 --dist --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c5y8_dist.json 2> $OUT/c5y8_dist.err || { echo "c5y8 failed"; tail -5 $OUT/c5y8_dist.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c5y8_dist.json')); print('c5y8', round(d['value']), 'MG', d['solve_time_s'], d['solve_iters'], d['ranks'])"
for t in 64 32; do
  LSQ_E_TILE=$t timeout -k 10 500 python3 -u tools/compute_e_at.py c4 > $OUT/compute_e_c4_t$t.json 2> $OUT/compute_e_c4_t$t.err || { echo "compute_E t=$t failed"; tail -5 $OUT/compute_e_c4_t$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/compute_e_c4_t$t.json')); print('t=$t', round(d['wall_s'],1), d['timing']['E_window'])"
done
