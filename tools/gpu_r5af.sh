# round 5: update kernel with one read per factor entry and a tight factor-word count
# (96 VGPRs, occupancy 5) — the full GPU suite, then the c4 bench three times
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5af}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/b$i.json 2> $OUT/b$i.err || { echo "bench failed"; tail -3 $OUT/b$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()}, r['frac'])"
done
