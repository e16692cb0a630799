"""GPU parity of the CGNR path (lsq_opts.method = 1; lsqr_cg.inc): the fused normal-stencil
operator must equal AᵀA of the formed (reference-identical) A, and PCG on the normal equations
must reach the exact LS solution within DESIGN.md's tolerance (||x-x*||/||x*|| <= 1e-6,
max|x-x*| <= 1e-4 m)."""
import numpy as np
import pytest

import lssurf_amd as LS
from conftest import SYSTEMS, golden, golden_csr, golden_kwargs, golden_points
from lssurf_amd.constraint_functions import reference_epoch_keep_cols
from lssurf_amd.smooth_fit import FitSystem

pytestmark = pytest.mark.gpu
REL, ABS = 1e-6, 1e-4
TOL = dict(atol=1e-12, btol=1e-12, conlim=1e12)


def _golden_system(name):
    g = golden(f'sys_{name}.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    w = 1. / np.sqrt((1 / (1. / np.concatenate((S['Ed'], S['Ec'])))) ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    return g, fs, w, rhs


def _synthetic_system(name='t64', stiff=False):
    from lssurf_amd import synthetic
    D, kw = synthetic.points(name)
    if stiff:
        kw['E_RMS'] = dict(synthetic.E_RMS_STIFF)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    w = 1. / np.sqrt((1 / (1. / np.concatenate((S['Ed'], S['Ec'])))) ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    return S, fs, w, rhs


@pytest.mark.parametrize('which', ['sf3d', 'nb_xt', 't64', 't256', 'tdense', 't15'])
def test_normal_operator_equals_assembled_normal_matrix(gpu_available, which):
    """q = N p from the class-coefficient stencil + Adᵀ(Ad p) equals Aᵀ(A p) computed with the
    formed A (bit-identical to the reference's matrix) on random p, every column incl. the
    boundary classes; removed (reference-epoch) columns carry p = 0.  t256 has dim-1 tiles clear
    of both edges (the wave-uniform coefficient path); the small grids only edge tiles."""
    if which in ('t64', 't256', 'tdense', 't15'):
        S, fs, w, rhs = _synthetic_system(which)
    else:
        g, fs, w, rhs = _golden_system(which)
    rng = np.random.default_rng(7)
    keep = rng.random(fs.n_data) > 0.2            # a row mask on data rows, as the editing loop sets
    try:
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.concatenate([keep, np.ones(fs.n_con, bool)]))
        ok, why = fs.solver.cg_available(1)
        assert ok, why
        A = fs.solver.get_csr()                   # selected rows, weighted, compact columns
        for _ in range(2):
            pc = rng.standard_normal(A.shape[1])
            pf = np.zeros(fs.n_full)
            pf[fs.keep_cols] = pc
            q = fs.solver.normal_apply(pf)[fs.keep_cols]
            qr = A.T @ (A @ pc)
            err = np.abs(q - qr).max() / np.abs(qr).max()
            assert err <= 1e-12, err
    finally:
        fs.close()


@pytest.mark.parametrize('precond', [3, 1])
@pytest.mark.parametrize('name', SYSTEMS)
def test_cgnr_matches_exact_solution(gpu_available, name, precond):
    g, fs, w, rhs = _golden_system(name)
    try:
        x = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=precond, method=1, maxit=200000, **TOL)
        st = fs.stats
    finally:
        fs.close()
    xs = g['x']
    assert st['method'] == 1, st
    assert st['istop'] in (1, 2), st
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) <= REL
    assert np.max(np.abs(x - xs)) <= ABS


def test_cgnr_tracks_lsqr_iterations_and_estimates(gpu_available):
    """Same Krylov space as LSQR on A·M^{-1/2}: comparable iteration counts, equal solutions,
    and the Lanczos-derived estimates (‖r‖, ‖Aᵀr‖ → 0, ‖A‖) agree with LSQR's at the end."""
    S, fs, w, rhs = _synthetic_system()
    keep = np.ones(fs.n_data, bool)
    try:
        out = {}
        for meth in (0, 1):
            x = fs.solve(w, keep, rhs, precond=3, method=meth, **TOL)
            out[meth] = (x, dict(fs.stats))
    finally:
        fs.close()
    (x0, s0), (x1, s1) = out[0], out[1]
    assert s0['method'] == 0 and s1['method'] == 1
    assert np.linalg.norm(x1 - x0) / np.linalg.norm(x0) <= 1e-8
    assert abs(s1['iters'] - s0['iters']) <= max(5, 0.1 * s0['iters']), (s0['iters'], s1['iters'])
    assert abs(s1['r1norm'] - s0['r1norm']) <= 1e-6 * s0['r1norm']
    assert abs(s1['anorm'] - s0['anorm']) <= 0.05 * s0['anorm']


def test_cgnr_mask_reweight_warm_start(gpu_available):
    S, fs, w, rhs = _synthetic_system()
    rng = np.random.default_rng(3)
    keep = rng.random(fs.n_data) > 0.1
    w2 = w * np.where(np.arange(w.size) < fs.n_data, rng.uniform(0.5, 2, w.size), 1.0)
    try:
        xl = fs.solve(w2, keep, rhs, precond=3, method=0, **TOL)
        x1 = fs.solve(w2, keep, rhs, precond=3, method=1, **TOL)
        it_cold = fs.stats['iters']
        x2 = fs.solve(w2, keep, rhs, x0=x1 * (1 + 1e-3), precond=3, method=1, **TOL)
        it_warm = fs.stats['iters']
        xj = fs.solve(w2, keep, rhs, precond=1, method=1, **TOL)
    finally:
        fs.close()
    for x in (x1, x2, xj):
        assert np.linalg.norm(x - xl) / np.linalg.norm(xl) <= 1e-8
    assert it_warm < it_cold


def test_cgnr_stiff_block_jacobi(gpu_available):
    """Stiff E_RMS (SURVEY.md §8(d) stress variant): block-Jacobi CGNR still reaches LSQR's
    solution."""
    S, fs, w, rhs = _synthetic_system(stiff=True)
    keep = np.ones(fs.n_data, bool)
    try:
        xl = fs.solve(w, keep, rhs, precond=3, method=0, **TOL)
        xc = fs.solve(w, keep, rhs, precond=3, method=1, **TOL)
        st = fs.stats
    finally:
        fs.close()
    assert st['method'] == 1 and st['istop'] in (1, 2), st
    assert np.linalg.norm(xc - xl) / np.linalg.norm(xl) <= 1e-7


def test_cgnr_falls_back_on_assembled_systems(gpu_available):
    g = golden('sys_sf3d.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, structured=False)
    w = 1. / np.sqrt((1 / (1. / np.concatenate((S['Ed'], S['Ec'])))) ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    try:
        ok, why = fs.solver.cg_available(1)
        x = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=1, method=1, **TOL)
        st = fs.stats
    finally:
        fs.close()
    assert not ok and why
    assert st['method'] == 0
    assert np.linalg.norm(x - g['x']) / np.linalg.norm(g['x']) <= REL


def test_smooth_fit_cgnr_default(gpu_available):
    """smooth_fit with the iterative path forced (lsq_precond=3): method 'auto' runs CGNR and the
    outputs match the reference's golden fit."""
    g = golden('sys_sf3d.npz')
    out = LS.smooth_fit(data=golden_points(g), lsq_precond=3, **golden_kwargs(g))
    assert out['timing']['lsq_last']['method'] == 1
    for got, ref in ((out['m']['z0'].z0, g['z0']), (out['m']['dz'].dz, g['dz']), (out['data'].z_est, g['data_z_est'])):
        ok = np.isfinite(ref)
        assert np.linalg.norm(got[ok] - ref[ok]) / np.linalg.norm(ref[ok]) < 1e-6
    assert np.nanmax(np.abs(out['m']['dz'].dz - g['dz'])) < ABS


def _lin2d_structured(g):
    """tests/golden sys_lin2d (the notebook's 2-D z0-only system, C2's structure) rebuilt with
    lssurf_amd.lin_op from the golden inputs and formed as a STRUCTURED system (lazy lin_op parts)."""
    from lssurf_amd.fd_grid import fd_grid
    from lssurf_amd.lin_op import lin_op
    grid = fd_grid([[0., 2300.], [0., 2300.]], [100., 100.], name='z0')
    G = lin_op(grid, name='interp_z').interp_mtx([g['in_y'], g['in_x']])
    root = np.sqrt(np.prod(grid.delta))
    g2 = lin_op(grid, name='grad2_z0').grad2(DOF='z0')
    g2.expected = 0.03 / root * np.ones(g2.N_eq)
    g1 = lin_op(grid, name='grad_z0').grad(DOF='z0')
    g1.expected = 75. / root * np.ones(g1.N_eq)
    Gc = lin_op(None, name='constraints').vstack([g2, g1])
    w = 1. / np.concatenate([g['in_sigma'], g2.expected, g1.expected])
    rhs = np.concatenate([g['in_z'], np.zeros(Gc.N_eq)])
    fs = FitSystem(G, Gc, np.arange(G.col_N), G.col_N, grids={'z0': grid})
    return fs, w, rhs


def test_cgnr_2d_lin_op_system_exact_solution(gpu_available):
    """C2 structure (2-D z0 grid, 1 node along dim 2: the MAXT = 1 column kernel): the lin_op
    system forms as a structured system, its normal operator equals the formed AᵀA, and CGNR
    (Jacobi) reaches the golden exact solution."""
    g = golden('sys_lin2d.npz')
    fs, w, rhs = _lin2d_structured(g)
    try:
        assert fs.formation == 'stencil'
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.ones(w.size, bool))
        ok, why = fs.solver.cg_available(1)
        assert ok, why
        A = fs.solver.get_csr()
        Ag = golden_csr(g)
        assert abs(A - Ag).max() <= 1e-12 * abs(Ag).max()
        rng = np.random.default_rng(3)
        p = rng.standard_normal(A.shape[1])
        q = fs.solver.normal_apply(p)
        qr = A.T @ (A @ p)
        assert np.abs(q - qr).max() <= 1e-12 * np.abs(qr).max()
        x = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=1, method=1, maxit=200000, **TOL)
        st = fs.stats
    finally:
        fs.close()
    assert st['method'] == 1 and st['istop'] in (1, 2), st
    xs = g['x']
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) <= REL
    assert np.max(np.abs(x - xs)) <= ABS


@pytest.mark.parametrize('which', ['t64', 'tdense', 't15', 'nb_xt'])
def test_matrix_free_data_rows_match_stored_rows(gpu_available, which, monkeypatch):
    """CGNR's matrix-free data rows (point subscripts sorted by cell, k_cg_dmf_*) against the
    stored Ad / ATd path (LSQ_CG_DMF=0, read at formation): same AᵀA p to rounding, same solve."""
    out = {}
    for flag in ('1', '0'):
        monkeypatch.setenv('LSQ_CG_DMF', flag)
        if which in ('t64', 'tdense', 't15'):
            S, fs, w, rhs = _synthetic_system(which)
        else:
            g, fs, w, rhs = _golden_system(which)
        keep = np.random.default_rng(5).random(fs.n_data) > 0.2
        try:
            fs.solver.set_row_weight(w)
            fs.solver.set_row_mask(np.concatenate([keep, np.ones(fs.n_con, bool)]))
            pf = np.zeros(fs.n_full)
            pf[fs.keep_cols] = np.random.default_rng(9).standard_normal(fs.keep_cols.size)
            q = fs.solver.normal_apply(pf)[fs.keep_cols]
            mode = fs.solver.profile_cg(reps=1)['data_rows']
            x = fs.solve(w, keep, rhs, precond=3, method=1, **TOL)
            out[flag] = (q, x, fs.stats['iters'], mode)
        finally:
            fs.close()
    (q1, x1, i1, m1), (q0, x0, i0, m0) = out['1'], out['0']
    assert m0 == 'stored' and (m1 == 'matrix-free' or which == 'nb_xt'), (m1, m0)
    assert np.abs(q1 - q0).max() <= 1e-12 * np.abs(q0).max()
    assert np.linalg.norm(x1 - x0) <= 1e-9 * np.linalg.norm(x0)
    assert abs(i1 - i0) <= 2, (i1, i0)
