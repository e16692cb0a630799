# does the bench command crash without the profiler / with the default output format? (development)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-prof_check}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/plain.json 2> $OUT/plain.err
echo "plain rc=$?"
[ -s $OUT/plain.json ] || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 200 --warmup 20 > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
