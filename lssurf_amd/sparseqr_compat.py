"""Drop-in for PySPQR's ``sparseqr.solve`` (used directly by notebooks/smooth_fit_demo_aniso.ipynb
cells 6, 13, 16, 18, 20 and by LSsurf/smooth_fit.py:142).

``solve(A, b, tolerance=None)`` returns the least-squares solution x (1-D, length n for 1-D b)
computed by device LSQR to a tight tolerance (atol = btol = 1e-12 by default) instead of a
sparse QR factorisation.  A full-column-rank A has a unique solution, so results agree with
SuiteSparseQR to the tolerance in DESIGN.md §Parity.  ``tolerance`` (SPQR's rank tolerance)
has no LSQR meaning and is ignored.  ``import lssurf_amd.sparseqr_compat as sparseqr``.
"""
import numpy as np
import scipy.sparse as sp

from .solver import LSQSolver

_DEFAULTS = dict(atol=1e-12, btol=1e-12, conlim=1e12, precond=1)


def solve(A, b, tolerance=None, device=0, **opts):
    A = sp.coo_matrix(A)
    b = np.asarray(b, dtype=np.float64)
    if b.ndim != 1:
        cols = [solve(A, b[:, k], tolerance, device, **opts) for k in range(b.shape[1])]
        return np.stack(cols, axis=1)
    kw = dict(_DEFAULTS, **opts)
    with LSQSolver(device) as s:
        s.set_matrix_coo(A.shape[0], A.shape[1], A.row, A.col, A.data)
        x, stats = s.solve(b, **kw)
    solve.last_stats = stats
    return x


solve.last_stats = None


def rz(A, b, tolerance=None, device=0):
    raise NotImplementedError('sparseqr.rz: use lssurf_amd.errors (normal-equation R on the device)')
