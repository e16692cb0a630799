# round 5: Ad·p with 1 / 2 (default) / 4 points per thread and trip (DMF_AD_U, tools/build_variant.sh)
# — the CGNR / multigrid GPU tests on the default build, then c4 CG steps alternating the builds
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5av}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cgnr.py tests/test_gpu_mg.py tests/test_gpu_aniso.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cp lssurf_amd/liblsqsurf.so tools/ab/lib_adu2.so
for i in 1 2; do
  for v in adu2 adu1 adu4; do
    cp tools/ab/lib_$v.so lssurf_amd/liblsqsurf.so
    timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 300 --warmup 20 > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || { echo "bench $v failed"; tail -3 $OUT/${v}_$i.err; cp tools/ab/lib_adu2.so lssurf_amd/liblsqsurf.so; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), {k: round(v*1e3,1) for k,v in r['kernel_ms'].items()})"
  done
done
cp tools/ab/lib_adu2.so lssurf_amd/liblsqsurf.so
