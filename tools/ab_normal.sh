# GPU-box A/B of liblsqsurf.so builds on the C4 normal-stencil role (development): each variant's
# bench line (--no-solve), then the base build with the stencil compute skipped (LSQ_CG_DBG=1:
# the kernel's memory floor; results wrong) and the ring kernel (LSQ_CG_RW=0)
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab_normal_${1}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --config c4 --no-cpu --no-pmc --no-solve --steps 100 --warmup 10 > $OUT/$n.json 2> $OUT/$n.err
  python3 -c "import json,sys; d=json.load(open('$OUT/$n.json')); print('$n', d['config'].get('normal_kernel'), round(d['value']), {k: round(v*1e3,1) for k,v in d['roofline']['kernel_ms'].items()})"
}
for i in 1 2; do
  for lib in "$@"; do
    cp tools/ab/lib_$lib.so lssurf_amd/liblsqsurf.so
    run ${lib}_$i X=1
  done
done
cp tools/ab/lib_$1.so lssurf_amd/liblsqsurf.so
run dbg1 LSQ_CG_DBG=1
run ring LSQ_CG_RW=0
echo ok > $OUT/ok
