# round 4 (development): the probing estimator of diag((AᵀA)⁻¹) on multigrid PCG against the band
# covariance at t64 (64²×12) and t128 (128²×12): VERDICT r3 #8 (the D = 16 pass at t64 ran past the
# 500 s limit — 0.18 s per probe through the host round trips — after D = 4 and 8 had reported)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4pr}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/probe_diag.py t64 4,8,16 0.127 > $OUT/probe_t64.jsonl 2> $OUT/probe_t64.err || { echo "t64 failed"; tail -5 $OUT/probe_t64.err; exit 1; }
grep -v "^\.\.\." $OUT/probe_t64.jsonl
timeout -k 10 500 python3 -u tools/probe_diag.py t128 4,8 0.127 > $OUT/probe_t128.jsonl 2> $OUT/probe_t128.err || { echo "t128 failed"; tail -5 $OUT/probe_t128.err; exit 1; }
grep -v "^\.\.\." $OUT/probe_t128.jsonl
