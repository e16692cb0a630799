# round 3: full GPU suite + C4 bench line (LSQR structured-operator regression check)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3c}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --config c4 --no-pmc --no-cpu --steps 200 --warmup 20 > $OUT/c4.json 2> $OUT/c4.err || echo "c4 rc=$?" >> $OUT/c4.err
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
echo "rc=$?" >> $OUT/tests.log
tail -3 $OUT/tests.log
python3 -c "import json;d=json.load(open('$OUT/c4.json'));print(d['value'],d['solve_time_s'],d['solve_lsqr'])"
