"""oracle/cgnr_cpu.c (TEST INFRASTRUCTURE: bench.py's algorithm-matched CPU baseline) against a
numpy restatement of block-Jacobi PCG on the normal equations, iterate for iterate, and against the
exact least-squares solution — on random systems and on the golden sys_sf3d (the reference's own
A and b, the smooth_fit node blocks)."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden, golden_csr
from oracle import cpu


def _pcg_numpy(A, b, blocks, iters):
    bp, bc = blocks
    N = (A.T @ A).toarray()
    Minv = np.zeros_like(N)
    for k in range(bp.size - 1):
        c = bc[bp[k]:bp[k + 1]]
        Minv[np.ix_(c, c)] = np.linalg.inv(N[np.ix_(c, c)])
    x = np.zeros(A.shape[1])
    s = A.T @ b
    z = Minv @ s
    p = z.copy()
    rho = s @ z
    for _ in range(iters):
        t = A @ p
        alpha = rho / (t @ t)
        x += alpha * p
        s -= alpha * (A.T @ t)
        z = Minv @ s
        rho2 = s @ z
        p = z + (rho2 / rho) * p
        rho = rho2
    return x


def _random(seed, m=500, n=72, k=12):
    rng = np.random.default_rng(seed)
    A = sp.random(m, n, density=0.08, random_state=rng, format='csr') + sp.eye(m, n, format='csr')
    b = rng.standard_normal(m)
    perm = rng.permutation(n)
    bp = np.arange(0, n + 1, k, dtype=np.int64)
    return sp.csr_matrix(A), b, (bp, perm.astype(np.int32))


def test_cgnr_bj_matches_numpy_pcg_iterates():
    A, b, blocks = _random(1)
    for iters in (1, 5, 20):
        x, st = cpu.cgnr_bj(A, b, *blocks, fixed_iters=iters, threads=2)
        assert int(st['iters']) == iters
        xr = _pcg_numpy(A, b, blocks, iters)
        assert np.linalg.norm(x - xr) <= 1e-10 * np.linalg.norm(xr)


def test_cgnr_bj_solves_to_the_least_squares_solution():
    A, b, blocks = _random(2)
    x, st = cpu.cgnr_bj(A, b, *blocks, atol=1e-14, maxit=500, threads=2)
    xs = np.linalg.lstsq(A.toarray(), b, rcond=None)[0]
    assert np.linalg.norm(x - xs) <= 1e-9 * np.linalg.norm(xs), st


def test_cgnr_bj_golden_system_with_node_blocks():
    import lssurf_amd as LS
    from conftest import golden_kwargs, golden_points
    from lssurf_amd.constraint_functions import node_column_blocks, reference_epoch_keep_cols
    g = golden('sys_sf3d.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    bp, bc = node_column_blocks(S['grids'], keep)
    A = golden_csr(g)
    x, st = cpu.cgnr_bj(A, g['b'], bp, bc, atol=1e-13, maxit=5000, threads=2)
    assert np.linalg.norm(x - g['x']) <= 1e-6 * np.linalg.norm(g['x']), st


def _golden_struct(name):
    import lssurf_amd as LS
    from conftest import golden_kwargs, golden_points
    from lssurf_amd.assemble import describe
    from lssurf_amd.constraint_functions import node_column_blocks, reference_epoch_keep_cols
    g = golden(f'sys_{name}.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    bp, bc = node_column_blocks(S['grids'], keep)
    w = 1. / np.sqrt((1 / (1. / np.concatenate((S['Ed'], S['Ec'])))) ** 2)
    desc = describe(S['G_data'], S['Gc'], with_fields=True)
    return g, S, keep, (bp, bc), w, desc


@pytest.mark.parametrize('name', ['sf3d', 't64'])
def test_cgnr_structured_kind_matches_csr_kind(name):
    """The structured CPU kind (oracle/cgnr_struct_cpu.c: stencil rows from the part descriptors,
    matrix-free data rows — the GPU line's operator, no stored matrix) runs the CSR kind's iteration:
    the same iterates to rounding after 1, 5 and 20 steps and the same iteration count to the
    stopping rule, on the golden system (the reference's own A and b) and on a synthetic system
    with z0 and dz on one lattice."""
    if name == 'sf3d':
        g, S, keep, blocks, w, desc = _golden_struct(name)
        A = golden_csr(g)
        b = g['b']
    else:
        import lssurf_amd as LS
        from lssurf_amd import synthetic
        from lssurf_amd.assemble import describe
        from lssurf_amd.constraint_functions import node_column_blocks, reference_epoch_keep_cols
        D, kw = synthetic.points('t64')
        S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
        keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
        blocks = node_column_blocks(S['grids'], keep)
        w = 1. / np.sqrt((1 / (1. / np.concatenate((S['Ed'], S['Ec'])))) ** 2)
        desc = describe(S['G_data'], S['Gc'], with_fields=True)
        G = sp.vstack([S['G_data'].toCSR(), S['Gc'].toCSR()]).tocsc()[:, keep]
        A = sp.csr_matrix(sp.diags(w) @ G)
        rhs = np.zeros(w.size)
        rhs[:S['data'].size] = S['data'].z
        b = w * rhs
    n_full = S['Gc'].col_N
    for iters in (1, 5, 20):
        xc, _ = cpu.cgnr_bj(A, b, *blocks, fixed_iters=iters, threads=2)
        xs, st = cpu.cgnr_bj_struct(desc, n_full, w, keep, b, *blocks, fixed_iters=iters, threads=2)
        assert int(st['iters']) == iters
        assert np.linalg.norm(xs - xc) <= 1e-10 * np.linalg.norm(xc), iters
    # to a rule above the rounding floor; PCG's ||s|| is not monotone, so summation-order rounding moves
    # the crossing by a few of t64's ~530 steps (golden: ±1)
    xc, stc = cpu.cgnr_bj(A, b, *blocks, atol=1e-11, maxit=5000, threads=2)
    xs, sts = cpu.cgnr_bj_struct(desc, n_full, w, keep, b, *blocks, atol=1e-11, maxit=5000, threads=2)
    assert abs(sts['iters'] - stc['iters']) <= (1 if name == 'sf3d' else 0.01 * stc['iters']), (sts, stc)
    assert abs(sts['anorm_f'] - stc['anorm_f']) <= 1e-10 * stc['anorm_f']
    assert np.linalg.norm(xs - xc) <= 1e-8 * np.linalg.norm(xc)
    if name == 'sf3d':
        xs, sts = cpu.cgnr_bj_struct(desc, n_full, w, keep, b, *blocks, atol=1e-13, maxit=5000, threads=2)
        assert np.linalg.norm(xs - g['x']) <= 1e-6 * np.linalg.norm(g['x']), sts
