# GPU-box check + A/B (development): the 8-wave normal-stencil kernel (LSQ_CG_W8=1) against the
# formed operator (CGNR / multigrid / distributed tests), then C4, C3, C1 and c4y8 with and without it
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-w8}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
LSQ_CG_W8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread > $OUT/tests_w8.log 2>&1
for i in 1 2; do
  for w in 0 1; do
    timeout -k 10 300 env LSQ_CG_W8=$w python3 bench.py --config c4 --no-cpu --no-pmc --steps 300 --warmup 20 > $OUT/c4_w${w}_$i.json 2> $OUT/c4_w${w}_$i.err
    timeout -k 10 300 env LSQ_CG_W8=$w python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --no-solve --steps 400 --warmup 20 > $OUT/c4y8_w${w}_$i.json 2> $OUT/c4y8_w${w}_$i.err
  done
done
for c in c3 c1; do
  for w in 0 1; do
    timeout -k 10 300 env LSQ_CG_W8=$w python3 bench.py --config $c --no-cpu --no-pmc --steps 300 --warmup 20 > $OUT/${c}_w$w.json 2> $OUT/${c}_w$w.err
  done
done
echo ok > $OUT/ok
