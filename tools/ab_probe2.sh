# normal-operator A/B (development): parity of the wave-strip path under each build (forced), then
# non-live role times and live bench lines, alternating
set -euo pipefail
cd $GRAFT_REPO_ROOT
for lib in "$@"; do
  cp tools/ab/lib_$lib.so lssurf_amd/liblsqsurf.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_normal_rw.py -x -q --timeout 280 --timeout-method thread 2>&1 | tail -1
done
for i in 1 2; do
  for lib in "$@"; do
    cp tools/ab/lib_$lib.so lssurf_amd/liblsqsurf.so
    echo -n "$lib: "; timeout -k 10 200 python3 tools/cg_phase_probe.py c4 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(d[k]*1e3,1) for k in ('cg_normal','cg_data','cg_update')})"
  done
done
cp tools/ab/lib_$1.so lssurf_amd/liblsqsurf.so
