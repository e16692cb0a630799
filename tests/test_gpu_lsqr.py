"""GPU parity of the solve path (through liblsqsurf's C ABI): device formation must equal the
reference's matrix bit-for-bit; LSQR must reach the exact LS solution within the stated
tolerance (||x-x*||/||x*|| <= 1e-6 and max|x-x*| <= 1e-4 m; the defaults
reach ~1e-9)."""
import numpy as np
import pytest
import scipy.sparse as sp

import lssurf_amd as LS
from conftest import SYSTEMS, golden, golden_csr, golden_kwargs, golden_points
from lssurf_amd.constraint_functions import reference_epoch_keep_cols
from lssurf_amd.smooth_fit import FitSystem
from oracle import cpu, dense

pytestmark = pytest.mark.gpu
REL, ABS = 1e-6, 1e-4


def _fit_system(name, structured=True):
    g = golden(f'sys_{name}.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    sysm = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, structured=structured)
    E_all = 1 / (1. / np.concatenate((S['Ed'], S['Ec'])))
    w = 1. / np.sqrt(E_all ** 2)
    rhs = np.zeros(S['G_data'].N_eq + S['Gc'].N_eq)
    rhs[:S['data'].size] = S['data'].z
    return g, S, sysm, w, rhs


@pytest.mark.parametrize('name', SYSTEMS)
@pytest.mark.parametrize('structured', [True, False])
def test_device_formation_bitwise(gpu_available, name, structured):
    g, S, sysm, w, rhs = _fit_system(name, structured)
    assert sysm.formation == ('stencil' if structured else 'coo')
    sysm.solver.set_row_weight(w)
    sysm.solver.set_row_mask(np.ones(sysm.n_data + sysm.n_con, bool))
    A = sysm.solver.get_csr()
    ref = golden_csr(g)
    sysm.close()
    assert A.shape == ref.shape
    np.testing.assert_array_equal(A.indptr, ref.indptr)
    np.testing.assert_array_equal(A.indices, ref.indices)
    np.testing.assert_array_equal(A.data, ref.data)


@pytest.mark.parametrize('name', SYSTEMS)
def test_lsqr_matches_exact_solution(gpu_available, name):
    g, S, sysm, w, rhs = _fit_system(name)
    x = sysm.solve(w, np.ones(sysm.n_data, bool), rhs, atol=1e-12, btol=1e-12, conlim=1e12)
    st = sysm.stats
    sysm.close()
    xs = g['x']
    assert st['istop'] in (1, 2), st
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) <= REL
    assert np.max(np.abs(x - xs)) <= ABS


@pytest.mark.parametrize('name', ['sf3d', 'nb_xt'])
def test_spmv_bitwise_vs_scipy(gpu_available, name):
    g, S, sysm, w, rhs = _fit_system(name)
    rng = np.random.default_rng(1)
    x = rng.normal(size=sysm.solver.n)
    y = sysm.solver.spmv(x)
    yt = sysm.solver.spmv(rng.normal(size=sysm.solver.m), trans=True)
    sysm.close()
    G = sp.vstack([S['G_data'].toCSR(), S['Gc'].toCSR()]).tocsr()
    G = sp.csr_matrix(G[:, sysm.keep_cols])
    G.sort_indices()
    np.testing.assert_array_equal(y, G.dot(x))
    assert yt.shape == (sysm.solver.n,)


def test_gpu_cpu_lsqr_agree(gpu_available):
    g = golden('sys_sf3d.npz')
    A = golden_csr(g)
    with LS.LSQSolver(0) as s:
        coo = A.tocoo()
        s.set_matrix_coo(A.shape[0], A.shape[1], coo.row, coo.col, coo.data)
        xg, stg = s.solve(g['b'], atol=1e-12, btol=1e-12, conlim=1e12)
    xc, stc = cpu.lsqr(A, g['b'], atol=1e-12, btol=1e-12, conlim=1e12)
    assert abs(stg['iters'] - stc['iters']) <= max(5, 0.05 * stc['iters'])
    assert np.linalg.norm(xg - xc) / np.linalg.norm(xc) < 1e-9


def test_row_mask_equals_row_removal(gpu_available):
    rng = np.random.default_rng(3)
    A = sp.random(400, 60, density=0.08, random_state=rng, format='csr') + sp.eye(400, 60)
    b = rng.normal(size=400)
    keep = rng.random(400) > 0.3
    w = rng.uniform(0.5, 2.0, 400)
    coo = A.tocoo()
    with LS.LSQSolver(0) as s:
        s.set_matrix_coo(400, 60, coo.row, coo.col, coo.data, row_weight=w)
        s.set_row_mask(keep)
        x1, _ = s.solve(b, atol=1e-13, btol=1e-13, conlim=1e14)
        Am = s.get_csr()
    Aref = sp.diags(w[keep]) @ A[keep]
    Aref = sp.csr_matrix(Aref)
    Aref.sort_indices()
    np.testing.assert_array_equal(Am.indices, Aref.indices)
    np.testing.assert_array_equal(Am.data, Aref.data)
    xs = dense.ls_solve_dense(Aref, w[keep] * b[keep])
    assert np.linalg.norm(x1 - xs) / np.linalg.norm(xs) < 1e-9


def test_duplicates_zeros_and_colmap(gpu_available):
    """toCSR semantics: drop v == 0, sum duplicates, drop zero sums, remove Ip_c columns."""
    rng = np.random.default_rng(4)
    m, n = 50, 30
    r = np.r_[rng.integers(0, m, 300), 5, 5, 5, 7, 7, 9]
    c = np.r_[rng.integers(0, n, 300), 3, 3, 3, 4, 4, 10**6]   # 3 dups, a cancelling pair, a bad col with v=0
    v = np.r_[rng.normal(size=300), 0.25, 0.5, 0.125, 1.5, -1.5, 0.0]
    v[::17] = 0.0
    keep_cols = np.setdiff1d(np.arange(n), [2, 11, 29])
    with LS.LSQSolver(0) as s:
        s.set_col_map(n, keep_cols)
        s.set_matrix_coo(m, n, r, c, v)     # the out-of-range column carries v == 0: ignored
        A = s.get_csr()
    nz = v != 0
    ref = sp.csr_matrix((v[nz], (r[nz], c[nz])), shape=(m, n))[:, keep_cols]
    ref = sp.csr_matrix(ref)
    ref.eliminate_zeros()
    ref.sort_indices()
    np.testing.assert_array_equal(A.indptr, ref.indptr)
    np.testing.assert_array_equal(A.indices, ref.indices)
    np.testing.assert_allclose(A.data, ref.data, rtol=1e-15)


def test_bad_index_raises(gpu_available):
    with LS.LSQSolver(0) as s:
        with pytest.raises(LS.solver.NativeError):
            s.set_matrix_coo(4, 4, np.array([0, 9]), np.array([0, 1]), np.array([1.0, 1.0]))


def test_warm_start_and_zero_rhs(gpu_available):
    g = golden('sys_lin2d.npz')
    A = golden_csr(g)
    coo = A.tocoo()
    with LS.LSQSolver(0) as s:
        s.set_matrix_coo(A.shape[0], A.shape[1], coo.row, coo.col, coo.data)
        x, st = s.solve(g['b'], atol=1e-12, btol=1e-12)
        x2, st2 = s.solve(g['b'], x0=x, atol=1e-12, btol=1e-12)
        z, stz = s.solve(np.zeros(A.shape[0]))
        x3, st3 = s.solve(g['b'], precond=0, atol=1e-12, btol=1e-12, conlim=1e14, maxit=20000)
        st_it = s.iterate(g['b'], 37)
    assert st2['iters'] < st['iters'] / 4
    assert np.linalg.norm(x2 - g['x']) / np.linalg.norm(g['x']) < 1e-8
    assert np.all(z == 0) and stz['iters'] == 0
    assert np.linalg.norm(x3 - g['x']) / np.linalg.norm(g['x']) < 1e-6
    assert st_it['iters'] == 37


def test_sparseqr_compat_solve(gpu_available):
    from lssurf_amd import sparseqr_compat as sparseqr
    g = golden('sys_lin2d.npz')
    x = sparseqr.solve(golden_csr(g).tocoo(), g['b'])
    assert x.ndim == 1
    assert np.linalg.norm(x - g['x']) / np.linalg.norm(g['x']) < 1e-8


def test_medium_system_formation_and_solve(gpu_available):
    """A 48x48x8 problem (bigger than the dense oracle likes): device formation == scipy
    formation bitwise; GPU LSQR == CPU oracle LSQR."""
    from lssurf_amd import containers as pc
    rng = np.random.default_rng(11)
    W = {'x': 4700., 'y': 4700., 't': 1.75}
    ctr = {'x': 0., 'y': 0., 't': 0.}
    n = 9000
    x = (rng.random(n) - .5) * W['x']
    y = (rng.random(n) - .5) * W['y']
    t = (rng.random(n) - .5) * W['t']
    z = 10 * np.sin(2 * np.pi * x / 2000) + t + rng.normal(0, .1, n)
    D = pc.data().from_dict({'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(n, .1)})
    kw = dict(W=W, ctr=ctr, spacing={'z0': 100., 'dz': 100., 'dt': .25},
              E_RMS={'d2z0_dx2': 0.03, 'dz0_dx': 75., 'd3z_dx2dt': 0.006, 'd2z_dxdt': 15., 'd2z_dt2': 5000.},
              reference_epoch=3, VERBOSE=False)
    S = LS.smooth_fit(data=D, return_fit_objects=True, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], 3)
    sysm = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N)
    E_all = 1 / (1. / np.concatenate((S['Ed'], S['Ec'])))
    wgt = 1. / np.sqrt(E_all ** 2)
    rhs = np.zeros(wgt.size)
    rhs[:S['data'].size] = S['data'].z
    xg = sysm.solve(wgt, np.ones(sysm.n_data, bool), rhs, atol=1e-12, btol=1e-12, conlim=1e12)
    A = sysm.solver.get_csr()
    sysm.close()
    N_eq = wgt.size
    G = sp.vstack([S['G_data'].toCSR(), S['Gc'].toCSR()]).tocoo()
    G = G.dot(LS.build_reference_epoch_matrix(S['G_data'], S['Gc'], S['grids'], 3))
    Aref = sp.csr_matrix(sp.dia_matrix((wgt, 0), shape=(N_eq, N_eq)).dot(G))
    Aref.sort_indices()
    np.testing.assert_array_equal(A.indices, Aref.indices)
    np.testing.assert_array_equal(A.data, Aref.data)
    xc, stc = cpu.lsqr(Aref, wgt * rhs, atol=1e-12, btol=1e-12, conlim=1e12)
    assert np.linalg.norm(xg - xc) / np.linalg.norm(xc) < 1e-8


@pytest.mark.parametrize('name', ['sf3d', 'nb_xt'])
def test_dense_preconditioned_lsqr(gpu_available, name):
    """precond 2 (device Cholesky R⁻¹ as right preconditioner): converges in a few iterations."""
    g, S, sysm, w, rhs = _fit_system(name)
    x = sysm.solve(w, np.ones(sysm.n_data, bool), rhs, atol=1e-14, btol=1e-14, conlim=1e16, precond=2)
    st = sysm.stats
    E = sysm.solver.sigma_x()
    Ri = sysm.solver.rinv()
    sysm.close()
    assert st['iters'] < 60, st
    assert np.linalg.norm(x - g['x']) / np.linalg.norm(g['x']) < 1e-10
    A = golden_csr(g)
    np.testing.assert_allclose(E, dense.diag_inv_normal(A), rtol=1e-8)
    R = np.linalg.inv(Ri)
    N = (A.T @ A).toarray()
    assert np.linalg.norm(R.T @ R - N) / np.linalg.norm(N) < 1e-12
    assert np.allclose(np.tril(Ri, -1), 0)


def test_dense_precond_stiff_kat_system(gpu_available):
    """The stiff notebook case (E_d2z0_dx2 = 0.0003, cond ~1e7) that column-scaled LSQR needs
    ~47 k iterations for."""
    from lssurf_amd import containers as pc
    k = golden('kat.npz')
    D = pc.data().from_dict({f[3:]: k[f] for f in k.files if f.startswith('in_')})
    E_RMS = {'d2z0_dx2': 0.0003, 'dz0_dx': 150., 'd3z_dx2dt': 0.0001, 'd2z_dxdt': 0.25, 'd2z_dt2': 5000}
    S = LS.smooth_fit(data=D, ctr={'x': 0., 'y': 0., 't': 0.}, W={'x': 1.e4, 'y': 200, 't': 2},
                      spacing={'z0': 50, 'dz': 100, 'dt': 0.25}, E_RMS=E_RMS, reference_epoch=2, VERBOSE=False,
                      return_fit_objects=True)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], 2)
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N)
    w = 1. / np.sqrt((1 / (1. / np.concatenate((S['Ed'], S['Ec'])))) ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    x = fs.solve(w, np.ones(fs.n_data, bool), rhs, atol=1e-14, btol=1e-14, conlim=1e16, precond=2)
    A = fs.solver.get_csr()
    fs.close()
    xs = dense.ls_solve_dense(A, w * rhs)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-9


def test_stencil_formation_equals_coo_formation_t64(gpu_available):
    """64x64x12, 8 k points: device-generated rows == host-triplet rows, bit for bit."""
    from lssurf_amd import synthetic
    D, kw = synthetic.points('t64')
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    mats = []
    for structured in (True, False):
        fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, structured=structured)
        mats.append(fs.solver.get_csr())
        fs.close()
    a, b = mats
    np.testing.assert_array_equal(a.indptr, b.indptr)
    np.testing.assert_array_equal(a.indices, b.indices)
    np.testing.assert_array_equal(a.data, b.data)


def _t64_system():
    from lssurf_amd import synthetic
    D, kw = synthetic.points('t64')
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N)
    E_all = 1 / (1. / np.concatenate((S['Ed'], S['Ec'])))
    w = 1. / np.sqrt(E_all ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    return S, fs, w, rhs


def test_stencil_operator_equals_assembled_operator(gpu_available):
    """The structured stencil operator (op 0) and the assembled SELL operator (op 1) run the same
    LSQR: after 40 fixed iterations the recurrence scalars agree to rounding, converged solutions
    to the solver tolerance."""
    S, fs, w, rhs = _t64_system()
    try:
        assert fs.solver.info()['stencil_op'] == 1
        fs.solver.set_row_weight(w)
        stats = [fs.solver.iterate(rhs, 40, op=op) for op in (0, 1)]
        for k in ('r1norm', 'anorm', 'arnorm', 'xnorm', 'acond'):
            assert abs(stats[0][k] - stats[1][k]) <= 1e-9 * abs(stats[1][k]), (k, stats)
        xs = [fs.solver.solve(rhs, atol=1e-12, btol=1e-12, conlim=1e12, op=op)[0] for op in (0, 1)]
    finally:
        fs.close()
    assert np.linalg.norm(xs[0] - xs[1]) / np.linalg.norm(xs[1]) <= 1e-8


def test_stencil_operator_mask_reweight_warm_start(gpu_available):
    S, fs, w, rhs = _t64_system()
    rng = np.random.default_rng(3)
    keep = rng.random(fs.n_data) > 0.1
    w2 = w * np.where(np.arange(w.size) < fs.n_data, rng.uniform(0.5, 2, w.size), 1.0)
    try:
        x0 = fs.solve(w2, keep, rhs, atol=1e-12, btol=1e-12, conlim=1e12, op=1)
        x1 = fs.solve(w2, keep, rhs, atol=1e-12, btol=1e-12, conlim=1e12, op=0)
        it_cold = fs.stats['iters']
        x2 = fs.solve(w2, keep, rhs, x0=x1, atol=1e-12, btol=1e-12, conlim=1e12, op=0)
        it_warm = fs.stats['iters']
    finally:
        fs.close()
    assert np.linalg.norm(x1 - x0) / np.linalg.norm(x0) <= 1e-8
    assert np.linalg.norm(x2 - x0) / np.linalg.norm(x0) <= 1e-8
    assert it_warm < it_cold


def _t64_blocks():
    from lssurf_amd import synthetic
    D, kw = synthetic.points('t64')
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    E_all = 1 / (1. / np.concatenate((S['Ed'], S['Ec'])))
    w = 1. / np.sqrt(E_all ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    return S, fs, w, rhs


@pytest.mark.parametrize('name', SYSTEMS)
def test_block_jacobi_matches_exact_solution(gpu_available, name):
    g = golden(f'sys_{name}.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    E_all = 1 / (1. / np.concatenate((S['Ed'], S['Ec'])))
    w = 1. / np.sqrt(E_all ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    try:
        assert fs.has_blocks
        x = fs.solve(w, np.ones(fs.n_data, bool), rhs, atol=1e-12, btol=1e-12, conlim=1e12, precond=3)
        st = fs.stats
    finally:
        fs.close()
    xs = g['x']
    assert st['istop'] in (1, 2), st
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) <= REL
    assert np.max(np.abs(x - xs)) <= ABS


def test_block_jacobi_both_operators_and_fewer_iterations(gpu_available):
    S, fs, w, rhs = _t64_blocks()
    keep = np.ones(fs.n_data, bool)
    tol = dict(atol=1e-12, btol=1e-12, conlim=1e12)
    try:
        x1 = fs.solve(w, keep, rhs, precond=1, **tol)
        it1 = fs.stats['iters']
        xb0 = fs.solve(w, keep, rhs, precond=3, op=0, **tol)
        itb0 = fs.stats['iters']
        xb1 = fs.solve(w, keep, rhs, precond=3, op=1, **tol)
        itb1 = fs.stats['iters']
        xw = fs.solve(w, keep, rhs, x0=xb0, precond=3, **tol)
        itw = fs.stats['iters']
    finally:
        fs.close()
    for x in (xb0, xb1, xw):
        assert np.linalg.norm(x - x1) / np.linalg.norm(x1) <= 1e-8
    assert abs(itb0 - itb1) <= max(3, 0.02 * itb0)
    assert itb0 < it1, (itb0, it1)
    assert itw < itb0


def test_column_blocks_validation(gpu_available):
    S, fs, w, rhs = _t64_blocks()
    try:
        with pytest.raises(Exception):
            fs.solver.set_column_blocks([np.arange(17)])          # too long
        with pytest.raises(Exception):
            fs.solver.set_column_blocks([[0, 1], [1, 2]])         # column in two blocks
        with pytest.raises(Exception):
            fs.solver.set_column_blocks([[0, 10 ** 9]])          # out of range
        fs.solver.set_column_blocks(None)                        # all singletons = Jacobi scaling
        x = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=3, atol=1e-12, btol=1e-12, conlim=1e12)
        x1 = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=1, atol=1e-12, btol=1e-12, conlim=1e12)
    finally:
        fs.close()
    assert np.linalg.norm(x - x1) / np.linalg.norm(x1) <= 1e-8


_CHILD_EPI = r'''
import sys, json
import numpy as np
sys.path.insert(0, sys.argv[1])
from test_gpu_lsqr import _t64_blocks
S, fs, w, rhs = _t64_blocks()
keep = np.ones(fs.n_data, bool)
tol = dict(atol=1e-12, btol=1e-12, conlim=1e12)
try:
    x = fs.solve(w, keep, rhs, precond=3, **tol)
    st = dict(fs.stats)
    xw = fs.solve(w, keep, rhs, x0=x * (1 + 1e-3), precond=3, **tol)
    stw = dict(fs.stats)
finally:
    fs.close()
np.savez(sys.argv[2], x=x, xw=xw)
print(json.dumps({'iters': int(st['iters']), 'iters_w': int(stw['iters']), 'bytes': float(st['bytes_per_iter'])}))
'''


def test_block_epilogue_lf_factor_bit_identical(gpu_available, tmp_path):
    """LSQR + block-Jacobi on the structured operator: the epilogue streaming the lf_t (bf16) factor
    copy gives x bit for bit equal to the f64-factor epilogue (LSQ_BLOCK_EPI_LF=0) — blk_Ri holds the
    rounded values, so both apply the same M — with the same iteration counts, cold and warm, and
    fewer algorithmic bytes per iteration.  Child processes (the switch is read once per process)."""
    import json
    import os
    import subprocess
    import sys
    out = {}
    for lf in ('1', '0'):
        path = tmp_path / f'x{lf}.npz'
        r = subprocess.run([sys.executable, '-c', _CHILD_EPI, os.path.dirname(__file__), str(path)],
                           env=dict(os.environ, LSQ_BLOCK_EPI_LF=lf), capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        out[lf] = (dict(np.load(path)), json.loads(r.stdout.strip().splitlines()[-1]))
    (a, sa), (b, sb) = out['1'], out['0']
    np.testing.assert_array_equal(a['x'], b['x'])
    np.testing.assert_array_equal(a['xw'], b['xw'])
    assert sa['iters'] == sb['iters'] and sa['iters_w'] == sb['iters_w'], (sa, sb)
    assert sa['bytes'] < sb['bytes'], (sa, sb)
