# round 5: identity sweeps with two listed tiles per workgroup (k_band_sweep_idn<2>: each R tile
# staged once for both) — the band / window / compute_E GPU tests, then compute_E at C3 and C4 with
# and without it (LSQ_BAND_NTL=1: k_band_sweep_id)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5at}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_band.py tests/test_gpu_errors_window.py tests/test_gpu_smooth_fit.py tests/test_gpu_rz.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for ntl in 2 1; do
  LSQ_BAND_NTL=$ntl timeout -k 10 300 python3 -u tools/compute_e_at.py c3 > $OUT/ce_c3_ntl$ntl.json 2> $OUT/ce_c3_ntl$ntl.err || { echo "compute_E c3 failed"; tail -5 $OUT/ce_c3_ntl$ntl.err; exit 1; }
  tail -1 $OUT/ce_c3_ntl$ntl.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['timing']['E_window']; print('c3 ntl=$ntl', round(d['wall_s'],1), round(e['time_s'],1), e['selfcheck_rel'], d['sigma_z0_sha16'])"
done
for ntl in 2 1; do
  LSQ_BAND_NTL=$ntl timeout -k 10 400 python3 -u tools/compute_e_at.py c4 > $OUT/ce_c4_ntl$ntl.json 2> $OUT/ce_c4_ntl$ntl.err || { echo "compute_E c4 failed"; tail -5 $OUT/ce_c4_ntl$ntl.err; exit 1; }
  tail -1 $OUT/ce_c4_ntl$ntl.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['timing']['E_window']; print('c4 ntl=$ntl', round(d['wall_s'],1), round(e['time_s'],1), e['selfcheck_rel'], d['sigma_z0_sha16'])"
done
