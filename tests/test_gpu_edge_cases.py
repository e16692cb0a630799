"""Edge cases of the solve boundary (lsq_set_matrix_coo / lsq_solve, sparseqr_compat.solve): empty
matrices, fully masked rows, empty columns and rows, a 1×1 system, one dense row over every column.
The expected results are scipy.sparse.linalg.lsqr's (the reference's LSQR semantics: x stays in
range(Aᵀ), so an empty column gets 0, and A = 0 or b = 0 stops at once with x = 0, istop 0) and
the dense exact least-squares solution of the oracle."""
import numpy as np
import pytest
import scipy.sparse as sp

import lssurf_amd as LS
from oracle import dense

pytestmark = pytest.mark.gpu
TOL = dict(atol=1e-13, btol=1e-13, conlim=1e14)


def _solve(A, b, row_weight=None, keep=None, **opts):
    coo = sp.coo_matrix(A)
    with LS.LSQSolver(0) as s:
        s.set_matrix_coo(A.shape[0], A.shape[1], coo.row, coo.col, coo.data, row_weight=row_weight)
        if keep is not None:
            s.set_row_mask(keep)
        return s.solve(b, **dict(TOL, **opts))


@pytest.mark.parametrize('precond', [0, 1])
def test_empty_matrix_gives_zero(gpu_available, precond):
    A = sp.csr_matrix((6, 4))
    b = np.arange(1.0, 7.0)
    x, st = _solve(A, b, precond=precond)
    assert x.shape == (4,) and np.all(x == 0)
    assert st['istop'] == 0 and st['iters'] == 0, st


def test_every_row_masked_gives_zero(gpu_available):
    rng = np.random.default_rng(1)
    A = sp.random(40, 10, density=0.3, random_state=rng, format='csr') + sp.eye(40, 10)
    x, st = _solve(A, rng.normal(size=40), keep=np.zeros(40, bool), precond=1)
    assert np.all(x == 0) and st['istop'] == 0, st


@pytest.mark.parametrize('precond', [0, 1])
def test_empty_columns_and_rows(gpu_available, precond):
    """Columns 2 and 7 have no entries (x = 0 there, LSQR's minimum-norm answer); rows 0, 5, 6
    have none either (they only add ‖b_i‖² to the residual)."""
    rng = np.random.default_rng(2)
    m, n = 60, 9
    A = sp.lil_matrix((m, n))
    for i in range(m):
        if i in (0, 5, 6):
            continue
        for j in rng.choice([0, 1, 3, 4, 5, 6, 8], size=3, replace=False):
            A[i, j] = rng.normal()
    A = A.tocsr()
    b = rng.normal(size=m)
    x, st = _solve(A, b, precond=precond)
    live = np.array([0, 1, 3, 4, 5, 6, 8])
    xs = np.zeros(n)
    xs[live] = dense.ls_solve_dense(sp.csr_matrix(A[:, live]), b)
    assert st['istop'] in (1, 2), st
    assert x[2] == 0 and x[7] == 0
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-9


def test_one_by_one(gpu_available):
    x, st = _solve(sp.csr_matrix(np.array([[2.0]])), np.array([4.0]), precond=0)
    assert st['istop'] in (1, 2) and abs(x[0] - 2.0) < 1e-14, (x, st)


def test_one_dense_row_over_every_column(gpu_available):
    """A ragged system: one row holds all n columns, the rest one entry each."""
    rng = np.random.default_rng(3)
    n = 3000
    A = sp.vstack([sp.csr_matrix(rng.uniform(0.5, 1.5, (1, n))), sp.diags(rng.uniform(1, 2, n))]).tocsr()
    b = rng.normal(size=n + 1)
    x, st = _solve(A, b, precond=1)
    xs = dense.ls_solve_dense(A, b)
    assert st['istop'] in (1, 2), st
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-9


def test_cgnr_on_an_assembled_system_reports_lsqr(gpu_available):
    """method 1 needs the structured normal operator: a COO system runs LSQR and says so."""
    rng = np.random.default_rng(4)
    A = sp.random(80, 20, density=0.2, random_state=rng, format='csr') + sp.eye(80, 20)
    b = rng.normal(size=80)
    x, st = _solve(A, b, precond=1, method=1)
    xs = dense.ls_solve_dense(A, b)
    assert st['method'] == 0 and st['istop'] in (1, 2), st
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-9


def test_sparseqr_compat_edge_cases(gpu_available):
    from lssurf_amd import sparseqr_compat as sparseqr
    rng = np.random.default_rng(5)
    A = (sp.random(50, 12, density=0.3, random_state=rng, format='csr') + sp.eye(50, 12)).tocoo()
    assert np.all(sparseqr.solve(A, np.zeros(50)) == 0)
    B = rng.normal(size=(50, 3))   # several right-hand sides: one solve per column, stacked
    X = sparseqr.solve(A, B)
    assert X.shape == (12, 3)
    for k in range(3):
        xs = dense.ls_solve_dense(sp.csr_matrix(A), B[:, k])
        assert np.linalg.norm(X[:, k] - xs) / np.linalg.norm(xs) < 1e-9
