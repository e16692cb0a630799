# GPU-box check (development): multigrid with the 8-wave level operator where strips do not fill
# the CUs — full GPU suite, then C1 / C3 solves with and without it (LSQ_CG_W8=0)
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-w8mg}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
for c in c1 c3; do
  for w in 0 d; do
    if [ $w = 0 ]; then E="LSQ_CG_W8=0"; else E="LSQ_CG_DUMMY=1"; fi
    timeout -k 10 300 env $E python3 bench.py --config $c --no-cpu --no-pmc --steps 300 --warmup 20 > $OUT/${c}_w$w.json 2> $OUT/${c}_w$w.err
  done
done
echo ok > $OUT/ok
