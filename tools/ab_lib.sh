# GPU-box A/B of builds of liblsqsurf.so (development): tools/ab/lib_base.so vs tools/ab/lib_<variant>.so for each variant argument,
# alternating, on C4 (bench + multigrid solve) and c4y8
set -euo pipefail
V="$*"; OUT=$GRAFT_REPO_ROOT/gpurun_out/ab_${1}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for lib in base $V; do
    cp tools/ab/lib_$lib.so lssurf_amd/liblsqsurf.so
    timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --steps 300 --warmup 20 > $OUT/c4_${lib}_$i.json 2> $OUT/c4_${lib}_$i.err
    timeout -k 10 300 python3 bench.py --config c4y8 --dist --no-cpu --no-pmc --no-solve --steps 400 --warmup 20 > $OUT/c4y8_${lib}_$i.json 2> $OUT/c4y8_${lib}_$i.err
  done
done
cp tools/ab/lib_base.so lssurf_amd/liblsqsurf.so
echo ok > $OUT/ok
