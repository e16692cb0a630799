set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3za}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for pw in 16 32 64; do
  LSQ_MG_PWG=$pw timeout -k 10 200 python3 -u tools/mg_trace.py c4 > $OUT/run_w$pw.log 2>&1 || exit 1; echo "pwg=$pw"; tail -1 $OUT/run_w$pw.log
done
for pm in 4096 1024; do
  LSQ_MG_PWG=32 LSQ_MG_PERSIST=$pm timeout -k 10 200 python3 -u tools/mg_trace.py c4 > $OUT/run_p$pm.log 2>&1 || exit 1; echo "pwg=32 persist=$pm"; tail -1 $OUT/run_p$pm.log
done
