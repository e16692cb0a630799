"""sparseqr.rz drop-in (lssurf_amd.sparseqr_compat.rz; LSsurf/smooth_fit.py:218): the device band
factor returned as SPQR's (Z, R, E, rank) — A[:, E] = Q·R with R upper triangular, Z = Qᵀb.
Checked on the reference's own smooth_fit matrix (sys_sf3d) and the anisotropic notebook
system: RᵀR = (A E)ᵀ(A E) to rounding, E·R⁻¹Z = the exact LS solution, and the reference's
error pipeline on R (inv_tr_upper → row RSS, smooth_fit.py:240-253) gives sqrt(diag((AᵀA)⁻¹))."""
import numpy as np
import pytest
import scipy.sparse as sp
from scipy.sparse.linalg import spsolve_triangular

from conftest import golden, golden_csr

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('name', ['sf3d', 'aniso37', 'aniso41', 'aniso3d'])
def test_rz_factor_and_solution(gpu_available, name):
    from lssurf_amd import sparseqr_compat as sq
    g = golden(f'sys_{name}.npz')
    A, b = golden_csr(g), g['b']
    Z, R, E, rank = sq.rz(A, b)
    n = A.shape[1]
    assert rank == n and R.shape == (n, n) and np.array_equal(np.sort(E), np.arange(n))
    assert sp.tril(R, -1).nnz == 0 and np.all(R.diagonal() > 0)
    AE = A[:, E]
    N = (AE.T @ AE).toarray()
    err = np.abs((R.T @ R).toarray() - N).max() / np.abs(N).max()
    assert err <= 1e-12, err
    y = spsolve_triangular(R.tocsr(), Z, lower=False)
    x = np.zeros(n)
    x[E] = y
    xs = g['x']
    # R is the Cholesky factor of the normal matrix: its forward error grows with cond(A)², which
    # the spread of R's diagonal bounds from below (sparseqr_compat.rz docstring)
    d = R.diagonal()
    tol = max(1e-9, 100 * np.finfo(float).eps * (d.max() / d.min()) ** 2)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) <= tol


def test_rz_feeds_the_reference_error_pipeline(gpu_available):
    """smooth_fit.py:240-253 on rz's R: inv_tr_upper (drop tolerance 1e-5, status retry loop), row
    RSS, un-permute by E — equals sqrt(diag((AᵀA)⁻¹)) to the drop tolerance."""
    import lssurf_amd as LS
    from lssurf_amd import sparseqr_compat as sq
    g = golden('sys_sf3d.npz')
    A, b = golden_csr(g), g['b']
    Z, R, E, rank = sq.rz(A, b)
    nnz_max = int(np.prod(R.shape) / 4)
    while True:
        RR, CC, VV, status = LS.inv_tr_upper(R.tocsr(), nnz_max, 1e-5)
        if status == 0:
            break
        nnz_max = int(nnz_max * 1.5)
    Rinv = sp.coo_matrix((VV, (E[RR], CC)), shape=R.shape).tocsr()
    E0 = np.sqrt(np.asarray(Rinv.power(2).sum(axis=1)).ravel())
    exact = np.sqrt(np.diag(np.linalg.inv((A.T @ A).toarray())))
    assert np.abs(E0 - exact).max() / exact.max() <= 1e-4
