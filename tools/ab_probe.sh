# non-live role times (tools/cg_phase_probe.py) of library variants, alternating (development)
set -euo pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for lib in "$@"; do
    cp tools/ab/lib_$lib.so lssurf_amd/liblsqsurf.so
    echo -n "$lib: "; timeout -k 10 200 python3 tools/cg_phase_probe.py c4 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(d[k]*1e3,1) for k in ('cg_normal','cg_data','cg_update')})"
  done
done
cp tools/ab/lib_$1.so lssurf_amd/liblsqsurf.so
