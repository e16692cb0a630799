# round 5: identity sweeps in column chunks (k_band_sweep_id<NC>) — error-propagation tests on the
# default build (NC = 32), then compute_E at 256²×12 (one lane) for NC = 64 / 32 / 16 and at C4
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5s}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_errors_window.py tests/test_gpu_band.py tests/test_gpu_rz.py tests/test_gpu_smooth_fit.py > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|^ERROR|^E  " $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
cp lssurf_amd/liblsqsurf.so /tmp/lib_default.so
for v in nc64 nc32 nc16; do
  cp tools/ab/lib_$v.so lssurf_amd/liblsqsurf.so
  LSQ_E_LANES=1 timeout -k 10 300 python3 tools/compute_e_at.py t256 > $OUT/ce_t256_$v.json 2> $OUT/ce_t256_$v.err || { echo "t256 $v failed"; tail -3 $OUT/ce_t256_$v.err; cp /tmp/lib_default.so lssurf_amd/liblsqsurf.so; exit 1; }
  tail -1 $OUT/ce_t256_$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['timing']['E_window']; print('t256 $v lanes=1', round(e['time_s'],2), e['selfcheck_rel'], d['sigma_z0_median'])"
done
cp /tmp/lib_default.so lssurf_amd/liblsqsurf.so
timeout -k 10 600 python3 -u tools/compute_e_at.py c4 > $OUT/ce_c4.json 2> $OUT/ce_c4.err || { echo "c4 failed"; tail -3 $OUT/ce_c4.err; exit 1; }
tail -1 $OUT/ce_c4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['timing']['E_window']; print('c4 nc32', round(d['wall_s'],1), round(e['time_s'],1), e['selfcheck_rel'], e['lanes'])"
