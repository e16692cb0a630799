# round 6: compute_E with the Schur window split — window tests, then C4 with the split (2 and 4
# lanes) and without it, σ saved for the comparison
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6c}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_errors_window.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/ewin_tests.log 2>&1 || { echo "window tests failed"; tail -40 $OUT/ewin_tests.log; exit 1; }
tail -3 $OUT/ewin_tests.log
LSQ_E_SAVE=/tmp/e_schur.npz timeout -k 10 400 python -u tools/compute_e_at.py c4 > $OUT/ce_c4_schur.json 2>&1 || { echo "c4 schur failed"; tail -20 $OUT/ce_c4_schur.json; exit 1; }
tail -1 $OUT/ce_c4_schur.json | cut -c1-900
LSQ_E_LANES=4 timeout -k 10 400 python -u tools/compute_e_at.py c4 > $OUT/ce_c4_schur_l4.json 2>&1 || { echo "c4 schur l4 failed"; tail -20 $OUT/ce_c4_schur_l4.json; exit 1; }
tail -1 $OUT/ce_c4_schur_l4.json | cut -c1-900
LSQ_E_SCHUR=0 LSQ_E_SAVE=/tmp/e_plain.npz timeout -k 10 400 python -u tools/compute_e_at.py c4 > $OUT/ce_c4_plain.json 2>&1 || { echo "c4 plain failed"; tail -20 $OUT/ce_c4_plain.json; exit 1; }
tail -1 $OUT/ce_c4_plain.json | cut -c1-600
python3 -c "
import numpy as np
a=np.load('/tmp/e_schur.npz'); b=np.load('/tmp/e_plain.npz')
for k in ('sigma_z0','sigma_dz'):
    x,y=a[k],b[k]; ok=np.isfinite(y)&(y>0)
    print(k, 'max rel', float(np.max(np.abs(x[ok]-y[ok])/y[ok])))
"
