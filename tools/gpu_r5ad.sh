# round 5: block factor read once per entry (lf_rowcol) — GPU tests of the CG / multigrid paths, then the c4 bench
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ad}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_aniso.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/b$i.json 2> $OUT/b$i.err || { echo "bench failed"; tail -3 $OUT/b$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), round(r['kernel_ms']['cg_update']*1e3,1), r['frac'])"
done
