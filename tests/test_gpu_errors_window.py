"""compute_E at scale: diag((AᵀA)⁻¹) by tiled windows (errors.window_cov,
lsq_cov_band_window) against the full band factor (lsq_cov_band) and the dense path.

* the full band factor is deterministic and equals the dense inverse at 64²×12 (≤ 1e-11) — a
  round-2 race in its sweeps (a workgroup's second step read the ring tile its first step had just
  written, without a barrier) made it differ by up to 100 % between calls at this size;
* tiles of 16 / 32 nodes with a 16 / 24-node margin: σ within 5e-4 / 1e-5 (max) of the full band
  at 64² / 128²×12 — the conditional variance given the columns outside the window, whose
  correlations with the tile decay with distance (DESIGN.md §Error propagation);
* averaging operators' errors through the windows (sys_avg golden system, tiles smaller than its
  grid, operators wider than a tile in windows of their own) within 1e-5 of the exact ones."""
import numpy as np
import pytest

import lssurf_amd as LS
from conftest import golden, golden_avg_masks, golden_kwargs, golden_points

pytestmark = pytest.mark.gpu


def _system(name, stiff=False):
    from lssurf_amd import synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    from lssurf_amd.smooth_fit import FitSystem
    D, kw = synthetic.points(name)
    if stiff:
        kw['E_RMS'] = dict(synthetic.E_RMS_STIFF)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    w = 1. / np.concatenate((S['Ed'], S['Ec']))
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.ones(w.size, bool))
    return S, fs, keep


def test_band_covariance_deterministic_and_exact(gpu_available):
    from lssurf_amd.errors import band_order
    S, fs, keep = _system('t64')
    try:
        o = band_order(S['grids'], keep)
        E1, _, _ = fs.solver.cov_band(o)
        E2, _, _ = fs.solver.cov_band(o)
        Ed = fs.solver.sigma_x()
    finally:
        fs.close()
    np.testing.assert_array_equal(E1, E2)
    assert np.max(np.abs(E1 - Ed) / Ed) <= 1e-11


@pytest.mark.parametrize('name,tile,margin,tol_max,tol_p99', [('t64', 16, 16, 5e-4, 3e-5),
                                                               ('t128', 32, 24, 1e-5, 1e-7)])
def test_window_covariance_matches_full_band(gpu_available, name, tile, margin, tol_max, tol_p99):
    """Measured (one box): margin 16 — max 7.6e-5 (64²) / 3.5e-4 (128²), 99th percentile 1.1e-5 /
    1.3e-5; margin 24 (the default) — max 3.1e-6, 99th percentile 7.8e-8 at 128²×12."""
    from lssurf_amd.errors import band_order, window_cov
    S, fs, keep = _system(name)
    try:
        Ef, _, _ = fs.solver.cov_band(band_order(S['grids'], keep))
        Ew, _, _ = window_cov(fs.solver, S["grids"], keep, tile=tile, margin=margin)
    finally:
        fs.close()
    rel = np.abs(Ew - Ef) / Ef
    assert rel.max() <= tol_max, rel.max()
    assert np.quantile(rel, 0.99) <= tol_p99, np.quantile(rel, 0.99)


def test_window_stiff_default_tile_and_self_check(gpu_available):
    """The stiff E_RMS (correlations reach further) with the default tile / margin (32 / 24 nodes):
    the window σ against the full band, and the self-check window_cov reports (the most central tile
    again with twice the margin) bounds the error it measures to within an order of magnitude —
    calc_and_parse_errors grows the margin when the self-check exceeds WINDOW_CHECK_TOL."""
    from lssurf_amd.errors import band_order, window_cov
    S, fs, keep = _system('t128', stiff=True)
    try:
        Ef, _, _ = fs.solver.cov_band(band_order(S['grids'], keep))
        Ew, _, check = window_cov(fs.solver, S['grids'], keep)
        Ew2, _, check2 = window_cov(fs.solver, S['grids'], keep, margin=48)
    finally:
        fs.close()
    rel = float(np.max(np.abs(Ew - Ef) / Ef))
    rel2 = float(np.max(np.abs(Ew2 - Ef) / Ef))
    print(f'stiff t128: margin 24 max rel {rel:.2e} (self-check {check:.2e}); margin 48 {rel2:.2e} ({check2:.2e})')
    assert np.isfinite(check) and check >= 0
    assert rel2 <= max(rel, 1e-12)              # a wider margin does not lose accuracy
    assert rel <= 20 * check + 1e-7, (rel, check)
    assert rel2 <= 2e-3, rel2


def test_window_averaging_errors(gpu_available):
    """smooth_fit(compute_E=True, lsq_E_method='window') with tiles smaller than the grid: the
    z0 / dz σ grids and the averaging products' errors against the reference's exact ones."""
    from lssurf_amd import errors
    g = golden('sys_avg.npz')
    saved = errors.WINDOW_TILE, errors.WINDOW_MARGIN
    errors.WINDOW_TILE, errors.WINDOW_MARGIN = 8, 16
    try:
        S = LS.smooth_fit(data=golden_points(g), avg_masks=golden_avg_masks(g), lsq_E_method='window',
                          **golden_kwargs(g))
    finally:
        errors.WINDOW_TILE, errors.WINDOW_MARGIN = saved
    assert S['timing']['E_window']['tiles'] > 1
    def rel(a, b):
        # explicit zero rule: entries where the reference is 0 (or NaN: cells outside the op's
        # output mask, NaN in both) must match exactly; the rest relative to |b|
        a, b = np.asarray(a, float), np.asarray(b, float)
        np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
        ok = np.isfinite(b)
        zero = ok & (b == 0)
        assert np.all(a[zero] == 0), 'non-zero error where the reference has 0'
        nz = ok & (b != 0)
        return float(np.max(np.abs(a[nz] - b[nz]) / np.abs(b[nz]))) if nz.any() else 0.0
    keys = [k[4:] for k in g.files if k.startswith('avg_')]
    for k in keys:
        E = getattr(S['E']['sigma_' + k], 'sigma_' + k)
        assert rel(E, g['Eexact_sigma_' + k]) < 1e-5, k


@pytest.mark.parametrize('lanes', ['1', '3'])
def test_batched_windows_equal_single_windows(gpu_available, lanes):
    """lsq_cov_band_windows (windows pipelined over stream lanes, interior-only sweeps, op rows as
    window positions) returns bit for bit what lsq_cov_band_window returns window by window: the
    same kernels in the same order per window, whatever runs beside it."""
    import os
    import scipy.sparse as sp
    from lssurf_amd.errors import band_order, _node_index
    S, fs, keep = _system('t64')
    saved = os.environ.get('LSQ_E_LANES')
    os.environ['LSQ_E_LANES'] = lanes
    try:
        o = band_order(S['grids'], keep)
        iy, ix = _node_index(S['grids'], keep)
        iy_o, ix_o = iy[o], ix[o]
        rng = np.random.default_rng(5)
        wins = []
        for (y0, x0) in [(0, 0), (16, 24), (40, 40), (8, 48)]:
            sel = np.flatnonzero((iy_o >= y0) & (iy_o < y0 + 24) & (ix_o >= x0) & (ix_o < x0 + 16))
            inner = (iy_o[sel] >= y0 + 4) & (iy_o[sel] < y0 + 20) & (ix_o[sel] >= x0 + 4) & (ix_o[sel] < x0 + 12)
            cols = o[sel]
            # op rows: pairs of the window's interior columns (as averaging operators' rows)
            a = rng.choice(cols[inner], size=70)
            b = rng.choice(cols[inner], size=70)
            op = sp.csr_matrix((np.r_[np.full(70, 0.5), np.full(70, 0.5)], (np.r_[np.arange(70), np.arange(70)],
                                np.r_[a, b])), shape=(70, keep.size))
            wins.append((cols, inner, op))
        Eb, ob, info = fs.solver.cov_band_windows(wins)
        for (cols, inner, op), e, oe in zip(wins, Eb, ob):
            es, oes, _ = fs.solver.cov_band_window(cols, op, inner=inner)
            np.testing.assert_array_equal(e, es)
            np.testing.assert_array_equal(oe, oes)
            assert np.all(e[~inner] == 0.0) and np.all(e[inner] > 0.0)
        assert int(info[5]) == int(lanes)
    finally:
        fs.close()
        if saved is None:
            os.environ.pop('LSQ_E_LANES', None)
        else:
            os.environ['LSQ_E_LANES'] = saved


def _golden_system(name):
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    from lssurf_amd.smooth_fit import FitSystem
    g = golden(f'sys_{name}.npz')
    kw = golden_kwargs(g)
    kw['VERBOSE'] = False
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    w = 1. / np.concatenate((S['Ed'], S['Ec']))
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.ones(w.size, bool))
    return S, fs, keep


@pytest.mark.parametrize('name,tile,margin', [('t128', 32, 24), ('sf3d_edit', 4, 3), ('deep1', 16, 8)])
def test_window_schur_split_equals_whole_window(gpu_available, name, tile, margin):
    """The Schur split (each window's bottom margin eliminated first, lsq_cov_band_windows_schur)
    is the same conditional variance as the whole window's band factor: equal to rounding, on the
    BASELINE layout (t128), z0 on a 2× refinement of the dz lattice (sf3d_edit) and the depth
    golden's lattice (deep1) — and its sweeps are fewer."""
    from lssurf_amd.errors import window_cov
    S, fs, keep = _golden_system(name) if name.startswith(('sf3d', 'deep')) else _system(name)
    try:
        t0, t1 = {}, {}
        Ew, _, c0 = window_cov(fs.solver, S['grids'], keep, tile=tile, margin=margin, schur=False, timing=t0)
        Es, _, c1 = window_cov(fs.solver, S['grids'], keep, tile=tile, margin=margin, schur=True, timing=t1)
    finally:
        fs.close()
    assert t1['E_window']['schur'] and not t0['E_window']['schur']
    assert np.all(Ew > 0)
    rel = np.abs(Es - Ew) / Ew
    assert rel.max() <= 1e-9, rel.max()
    assert abs(c1 - c0) <= 1e-9 + 1e-6 * abs(c0)
    assert t1['E_window']['tile_products'] < t0['E_window']['tile_products']


_CHILD_E = r'''
import sys, json
import numpy as np
sys.path.insert(0, sys.argv[1])
import lssurf_amd as LS
from lssurf_amd import synthetic
from lssurf_amd.constraint_functions import reference_epoch_keep_cols
from lssurf_amd.errors import window_cov
from lssurf_amd.smooth_fit import FitSystem
D, kw = synthetic.points('t128')
S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
w = 1. / np.concatenate((S['Ed'], S['Ec']))
fs.solver.set_row_weight(w)
fs.solver.set_row_mask(np.ones(w.size, bool))
try:
    E, _, c = window_cov(fs.solver, S['grids'], keep, tile=32, margin=24)
finally:
    fs.close()
np.save(sys.argv[2], E)
'''


def test_window_batches_bit_identical(gpu_available, tmp_path):
    """Windows factored in batches (one launch per step for LSQ_E_FBATCH windows, the default 8)
    give σ bit for bit equal to one window at a time (LSQ_E_FBATCH=1): the same kernels on the
    same bands.  Two child processes (the switch is read once per process)."""
    import os
    import subprocess
    import sys
    out = {}
    for fb in ('1', '8'):
        path = tmp_path / f'E{fb}.npy'
        r = subprocess.run([sys.executable, '-c', _CHILD_E, os.path.dirname(__file__), str(path)],
                           env=dict(os.environ, LSQ_E_FBATCH=fb), capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        out[fb] = np.load(path)
    np.testing.assert_array_equal(out['1'], out['8'])
    assert np.all(out['8'] > 0)
