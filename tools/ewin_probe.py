"""Development probe: tiled-window diag((AᵀA)⁻¹) (errors.window_cov) against the full band factor
(lsq_cov_band) on synthetic systems, per tile / margin; plus timing of the windowed path at C3."""
import json, sys, time
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import lssurf_amd as LS
from lssurf_amd import synthetic
from lssurf_amd.constraint_functions import reference_epoch_keep_cols
from lssurf_amd.errors import band_order, window_cov
from lssurf_amd.smooth_fit import FitSystem


def system(name):
    D, kw = synthetic.points(name)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    w = 1. / np.concatenate((S['Ed'], S['Ec']))
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.ones(w.size, bool))
    return S, fs, keep


def diag(name, tile, margin):
    from lssurf_amd.errors import _node_index
    S, fs, keep = system(name)
    Ef, _, info = fs.solver.cov_band(band_order(S['grids'], keep))
    Ew, _, _ = window_cov(fs.solver, S['grids'], keep, tile=tile, margin=margin)
    iy, ix = _node_index(S['grids'], keep)
    z0n = S['grids']['z0'].N_nodes
    nt = S['grids']['dz'].shape[2]
    rel = np.abs(Ew - Ef) / Ef
    Ewf, _, _ = window_cov(fs.solver, S['grids'], keep, tile=64, margin=0)   # one window = everything
    print('one-window vs full band max rel', float(np.max(np.abs(Ewf - Ef) / Ef)))
    if keep.size <= 60000:
        Ed = fs.solver.sigma_x()
        print('dense vs full band max rel', float(np.max(np.abs(Ed - Ef) / Ed)),
              'dense vs window max rel', float(np.max(np.abs(Ed - Ew) / Ed)))
        Ef = Ed
        rel = np.abs(Ew - Ef) / Ef
    worst = np.argsort(rel)[::-1][:12]
    for c in worst:
        full = keep[c]
        kind = 'z0' if full < z0n else 'dz t=%d' % ((full - z0n) % nt)
        print(json.dumps({'col': int(c), 'iy': int(iy[c]), 'ix': int(ix[c]), 'kind': kind, 'Ew': float(Ew[c]),
                          'Ef': float(Ef[c]), 'rel': float(rel[c])}))
    print('n bad > 1e-3:', int((rel > 1e-3).sum()), 'of', rel.size)
    fs.close()


if __name__ != '__main__':
    pass
elif sys.argv[1] == 'diag':
    diag(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    sys.exit(0)
for name in (sys.argv[1:] if __name__ == '__main__' else []):
    S, fs, keep = system(name)
    if name != 'c3':
        t0 = time.time()
        Ef, _, info = fs.solver.cov_band(band_order(S['grids'], keep))
        tf = time.time() - t0
        print(json.dumps({'name': name, 'full_band_s': tf, 'w': int(info[0])}), flush=True)
        combos = ((16, 4), (16, 8), (16, 12), (16, 16), (32, 16), (32, 24))
        if os.environ.get('EWIN_COMBOS'):
            combos = [tuple(int(v) for v in c.split('/')) for c in os.environ['EWIN_COMBOS'].split(',')]
        for tile, margin in combos:
            t0 = time.time()
            Ew, _, _ = window_cov(fs.solver, S["grids"], keep, tile=tile, margin=margin)
            rel = np.abs(Ew - Ef) / Ef
            worst = int(np.argmax(rel))
            print(json.dumps({'name': name, 'tile': tile, 'margin': margin, 'time_s': time.time() - t0,
                              'worst_col': worst, 'worst_Ew': float(Ew[worst]), 'worst_Ef': float(Ef[worst]),
                              'frac_low': float(np.mean(Ew < Ef)),
                              'max_rel': float(rel.max()), 'median_rel': float(np.median(rel)),
                              'p99_rel': float(np.quantile(rel, 0.99))}), flush=True)
    else:
        tm = {}
        t0 = time.time()
        Ew, _, _ = window_cov(fs.solver, S['grids'], keep, timing=tm)
        print(json.dumps({'name': name, 'n': int(keep.size), 'time_s': time.time() - t0, **tm,
                          'E_median': float(np.median(Ew)), 'E_min': float(Ew.min())}), flush=True)
    fs.close()
