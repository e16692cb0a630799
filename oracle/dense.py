"""Exact least-squares oracle (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

The reference solves ``argmin ||A x - b||`` with SuiteSparseQR through PySPQR
(``sparseqr.solve`` at LSsurf/smooth_fit.py:142, notebooks/smooth_fit_demo_aniso.ipynb
cells 6/13/16/18/20) and factors ``A = Q R E'`` with ``sparseqr.rz`` (smooth_fit.py:218).
PySPQR/SuiteSparse are external, unpinned (requirements.txt:7 is an unversioned git URL) and
absent offline.  For a full-column-rank A the least-squares solution is unique, so any exact
solver is a valid stand-in: here a dense Cholesky of AᵀA with corrected-semi-normal-equation
refinement (accuracy ~ eps*cond(A)), verified by the optimality residual ||Aᵀ(b-Ax)||.

``rz_dense`` returns the same tuple shape as ``sparseqr.rz``: (Z = Qᵀb, R (CSR, upper
triangular, columns permuted), E (column permutation), rank).
"""
import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp


def ls_solve_dense(A, b, refine=4):
    """Exact LS solution of a (modest-size) sparse system: x = argmin ||Ax-b||."""
    A = sp.csr_matrix(A)
    b = np.asarray(b, dtype=np.float64).ravel()
    N = (A.T @ A).toarray()
    c = sla.cho_factor(N, lower=False, check_finite=False)
    x = sla.cho_solve(c, A.T @ b, check_finite=False)
    for _ in range(refine):
        r = b - A @ x
        dx = sla.cho_solve(c, A.T @ r, check_finite=False)
        x = x + dx
        if np.max(np.abs(dx)) <= 1e-15 * max(1.0, np.max(np.abs(x))):
            break
    return x


def optimality(A, b, x):
    """||Aᵀ(b-Ax)|| / (||A||_F ||b-Ax||): ~eps for an exact LS solution."""
    r = b - A @ x
    g = A.T @ r
    return float(np.linalg.norm(g) / (sp.linalg.norm(A) * max(np.linalg.norm(r), 1e-300)))


def rz_dense(A, b):
    """Dense pivoted-QR stand-in for sparseqr.rz: returns (Z, R_csr, E, rank)."""
    Ad = sp.csr_matrix(A).toarray()
    Q, R, E = sla.qr(Ad, mode='economic', pivoting=True)
    Z = Q.T @ np.asarray(b, dtype=np.float64)
    d = np.abs(np.diag(R))
    rank = int(np.sum(d > d[0] * max(Ad.shape) * np.finfo(float).eps)) if d.size else 0
    R = sp.csr_matrix(np.triu(R))
    return Z, R, E, rank


def diag_inv_normal(A):
    """sqrt(diag((AᵀA)^-1)) — the quantity calc_and_parse_errors estimates (smooth_fit.py:253)."""
    N = (sp.csr_matrix(A).T @ sp.csr_matrix(A)).toarray()
    c = sla.cho_factor(N, lower=False)
    Ninv = sla.cho_solve(c, np.eye(N.shape[0]))
    return np.sqrt(np.diag(Ninv))
