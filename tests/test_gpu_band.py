"""GPU parity of the banded error propagation (lsq_cov_band, lssurf_amd/csrc/band.hip) — the
compute_E path that replaces sparseqr.rz + inv_tr_upper (smooth_fit.py:218-270).

* E = sqrt(diag((AᵀA)⁻¹)) equals the dense device factor's (lsq_sigma_x) and a host scipy
  inverse; masked rows and re-weighting included;
* op-row errors sqrt(diag(op (AᵀA)⁻¹ opᵀ)) equal the dense R⁻¹ products, for rows local to the
  band and rows spread over the whole grid;
* smooth_fit(compute_E=True) with the band path equals the dense path and the golden grids."""
import numpy as np
import pytest
import scipy.sparse as sp

import lssurf_amd as LS
from conftest import golden, golden_kwargs, golden_points
from lssurf_amd.errors import band_order
from test_gpu_cgnr import _golden_system

pytestmark = pytest.mark.gpu


def _prepare(fs, w, keep):
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.concatenate([keep, np.ones(fs.n_con, bool)]))


def _rel(a, b):
    return np.abs(a - b).max() / np.abs(b).max()


def _small_system(S=24, nt=12, seed=7):
    """smooth_fit system on an S×S×nt grid, 2 points per node (dense-comparable size)."""
    from lssurf_amd import synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    from lssurf_amd.smooth_fit import FitSystem
    W = {'x': (S - 1) * 100., 'y': (S - 1) * 100., 't': (nt - 1) * 0.25}
    rng = np.random.default_rng(seed)
    npts = 2 * S * S
    x, y = (rng.random(npts) - 0.5) * W['x'], (rng.random(npts) - 0.5) * W['y']
    t = (rng.random(npts) - 0.5) * W['t']
    z = 10 * np.sin(2 * np.pi * x / (W['x'] / 2)) + rng.normal(0, 0.1, npts)
    D = LS.containers.data().from_dict({'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(npts, 0.1)})
    out = LS.smooth_fit(data=D, W=W, ctr={'x': 0., 'y': 0., 't': 0.}, spacing={'z0': 100., 'dz': 100., 'dt': 0.25},
                        E_RMS=dict(synthetic.E_RMS_NOTEBOOK), reference_epoch=nt // 2, return_fit_objects=True)
    keep = reference_epoch_keep_cols(out['G_data'].col_N, out['grids']['dz'], nt // 2)
    fs = FitSystem(out['G_data'], out['Gc'], keep, out['Gc'].col_N, grids=out['grids'])
    w = 1. / np.concatenate((out['Ed'], out['Ec']))
    return out, fs, w


@pytest.mark.parametrize('which', ['s24', 's30t5', 'sf3d', 'nb_xt'])
def test_band_sigma_matches_dense(gpu_available, which):
    if which == 's24':
        S, fs, w = _small_system(24, 12)
        grids = S['grids']
    elif which == 's30t5':
        S, fs, w = _small_system(30, 5)
        grids = S['grids']
    else:
        g, fs, w, rhs = _golden_system(which)
        S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **golden_kwargs(g))
        grids = S['grids']
    rng = np.random.default_rng(3)
    keep = rng.random(fs.n_data) > 0.1
    try:
        _prepare(fs, w, keep)
        Ed = fs.solver.sigma_x()
        perm = band_order(grids, fs.keep_cols)
        Eb, _, info = fs.solver.cov_band(perm)
        Ei, _, info_i = fs.solver.cov_band(None)            # natural order: a (nearly) full band
        fs.solver.set_row_weight(w * 1.5)                   # re-weighting: a new factor
        Eb2, _, _ = fs.solver.cov_band(perm)
    finally:
        fs.close()
    assert info[0] < info[1] or info[1] <= 2, info       # node order: a real band
    assert _rel(Eb, Ed) < 1e-11, _rel(Eb, Ed)
    assert _rel(Ei, Ed) < 1e-11
    assert _rel(Eb2 * 1.5, Eb) < 1e-10


def test_band_sigma_matches_host_inverse(gpu_available):
    g, fs, w, rhs = _golden_system('sf3d')
    try:
        _prepare(fs, w, np.ones(fs.n_data, bool))
        A = fs.solver.get_csr()
        S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **golden_kwargs(g))
        Eb, _, _ = fs.solver.cov_band(band_order(S['grids'], fs.keep_cols))
    finally:
        fs.close()
    Aw = A                       # lsq_get_csr: the weighted, masked operator
    Ninv = np.linalg.inv((Aw.T @ Aw).toarray())
    assert _rel(Eb, np.sqrt(np.diag(Ninv))) < 1e-9


def test_band_op_rows_in_and_out_of_band(gpu_available):
    S, fs, w = _small_system(28, 12)
    rng = np.random.default_rng(9)
    n = fs.keep_cols.size
    perm = band_order(S['grids'], fs.keep_cols)
    pos = np.empty(n, int)
    pos[perm] = np.arange(n)
    rows, cols, vals = [], [], []
    for i in range(300):
        if i % 3 == 0:      # local: a few columns near one position (inside the band)
            c0 = rng.integers(0, n - 20)
            cc = perm[c0 + rng.choice(20, 4, replace=False)]
        elif i % 3 == 1:    # wide: columns far apart (outside the band)
            cc = rng.choice(n, 6, replace=False)
        else:               # single column
            cc = rng.choice(n, 1)
        rows += [i] * cc.size
        cols += list(cc)
        vals += list(rng.standard_normal(cc.size))
    op = sp.csr_matrix((vals, (rows, cols)), shape=(300, n))
    try:
        _prepare(fs, w, np.ones(fs.n_data, bool))
        E, oe, info = fs.solver.cov_band(perm, op)
        Ri = fs.solver.rinv()
    finally:
        fs.close()
    ref = np.sqrt(((op @ Ri) ** 2).sum(axis=1)).ravel()
    assert _rel(oe, ref) < 1e-11, _rel(oe, ref)
    single = np.diff(op.indptr) == 1
    assert _rel(oe[single], E[op.indices[op.indptr[:-1][single]]] * np.abs(op.data[op.indptr[:-1][single]])) < 1e-12


def test_band_rejects_bad_perm(gpu_available):
    from lssurf_amd._native import NativeError
    S, fs, w = _small_system(12, 6)
    try:
        _prepare(fs, w, np.ones(fs.n_data, bool))
        bad = np.zeros(fs.keep_cols.size, np.int32)
        with pytest.raises(NativeError):
            fs.solver.cov_band(bad)
    finally:
        fs.close()


def test_smooth_fit_compute_E_band_equals_dense(gpu_available):
    g = golden('sys_avg.npz')
    from conftest import golden_avg_masks
    out = {}
    for method in ('band', 'dense'):
        out[method] = LS.smooth_fit(data=golden_points(g), avg_masks=golden_avg_masks(g), lsq_E_method=method,
                                    **golden_kwargs(g))
    Eb, Ed = out['band']['E'], out['dense']['E']
    assert set(Eb) == set(Ed)
    for k in Ed:
        a, b = getattr(Eb[k], k), getattr(Ed[k], k)
        ok = np.isfinite(b)
        assert np.array_equal(ok, np.isfinite(a)), k
        assert _rel(a[ok], b[ok]) < 1e-10, k
    assert out['band']['timing']['E_band']['tiles'] >= 1


def test_band_empty_and_single_column_op_rows(gpu_available):
    """op rows with no entries give 0; a row with one entry gives |v|·E of its column."""
    S, fs, w = _small_system(10, 4)
    n = fs.keep_cols.size
    op = sp.csr_matrix((np.array([2.0, -3.0]), (np.array([1, 3]), np.array([0, n - 1]))), shape=(4, n))
    try:
        _prepare(fs, w, np.ones(fs.n_data, bool))
        E, oe, info = fs.solver.cov_band(band_order(S['grids'], fs.keep_cols), op)
    finally:
        fs.close()
    assert oe[0] == 0.0 and oe[2] == 0.0
    assert abs(oe[1] - 2.0 * E[0]) <= 1e-12 * E[0] and abs(oe[3] - 3.0 * E[n - 1]) <= 1e-12 * E[n - 1]
