# round 5 (development): the fused level-0 node gather + smoothing — grid A/B and its kernel trace
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5l}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "LSQ_MG_ATQ_GRID=1" "LSQ_MG_ATQ_GRID=0" "LSQ_MG_ATQ_SMOOTH=0"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/c4_$tag.json 2> $OUT/c4_$tag.err || { tail -5 $OUT/c4_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4_$tag.json')); print('c4 $v', round(d['value']), 'MG', round(d['solve_time_s'],4), d['solve_iters'])"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
python3 tools/mg_iter_trace.py $OUT/prof/run_kernel_trace.csv > $OUT/mg_iter_trace.txt && tail -25 $OUT/mg_iter_trace.txt
