"""GPU parity of the band preconditioner (precond 5: LSQR on A·P·S·R̃⁻¹, csrc/band.hip) and the
sparseqr.solve drop-in on the anisotropic notebook system (notebooks/smooth_fit_demo_aniso.ipynb
cells 13-18; BASELINE config C5's constraint)."""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from conftest import golden, golden_csr
from lssurf_amd import aniso
from lssurf_amd import sparseqr_compat as sparseqr
from lssurf_amd.solver import LSQSolver

pytestmark = pytest.mark.gpu


def _exact(A, b):
    """Host LS solution from the normal equations (sparse LU) + one refinement step."""
    A = sp.csr_matrix(A)
    N = (A.T @ A).tocsc()
    lu = spla.splu(N)
    x = lu.solve(A.T @ b)
    return x + lu.solve(A.T @ (b - A @ x))


def test_precond5_matches_dense_precond_on_golden(gpu_available):
    g = golden('sys_lin2d.npz')
    A = golden_csr(g).tocoo()
    with LSQSolver(0) as s:
        s.set_matrix_coo(A.shape[0], A.shape[1], A.row, A.col, A.data)
        x5, st5 = s.solve(g['b'], atol=1e-12, btol=1e-12, precond=5)
        x2, st2 = s.solve(g['b'], atol=1e-12, btol=1e-12, precond=2)
        xw, stw = s.solve(g['b'], x0=x5 * (1 + 1e-6), atol=1e-12, btol=1e-12, precond=5)   # warm start
    rel = lambda a: np.linalg.norm(a - g['x']) / np.linalg.norm(g['x'])
    assert st5['istop'] in (1, 2) and st5['iters'] <= 20, st5
    assert rel(x5) < 1e-9 and rel(x2) < 1e-9 and rel(xw) < 1e-9
    assert stw['iters'] <= st5['iters']


def test_precond5_with_an_order(gpu_available, monkeypatch):
    """A shuffled column order (bandwidth-reducing order passed by the caller): same solution."""
    monkeypatch.setattr(sparseqr, 'BAND_MAX_COLS', 300)   # force the reverse Cuthill-McKee order
    A, b, g = aniso.system(61, npts=500)
    rng = np.random.default_rng(1)
    shuffle = rng.permutation(A.shape[1])
    As = sp.csr_matrix(A)[:, shuffle].tocoo()          # columns scrambled: natural order is not banded
    perm, bw = sparseqr.band_order(As)
    assert perm is not None
    with LSQSolver(0) as s:
        s.set_matrix_coo(As.shape[0], As.shape[1], As.row, As.col, As.data)
        s.set_band_order(perm)
        x, st = s.solve(b, atol=1e-12, btol=1e-12, precond=5)
    xs = _exact(As, b)
    assert st['iters'] <= 30, st
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8


@pytest.mark.parametrize('nodes,npts', [(201, 0), (161, 50_000)])
def test_sparseqr_compat_aniso_notebook(gpu_available, nodes, npts):
    """The notebook's anisotropic system (8 points on a circle, or a dense cloud): column-scaled
    LSQR needs > 5·10⁴ iterations at the notebook's 401²; the band factor a few."""
    A, b, g = aniso.system(nodes, npts=npts)
    x = sparseqr.solve(A, b)
    st = sparseqr.solve.last_stats
    xs = _exact(A, b)
    assert st['istop'] in (1, 2) and st['iters'] <= 40, st
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-7


def test_precond5_row_mask_reweight_and_tiny_systems(gpu_available):
    """Row masks and re-weighting refactor the band (the factor follows the row scaling); a
    single-tile system (T = 1, w = 0) and a 2-tile one take the same code path."""
    for nodes in (5, 9, 61):
        A, b, g = aniso.system(nodes, npts=50)
        A = sp.csr_matrix(A)
        rng = np.random.default_rng(nodes)
        keep = rng.random(A.shape[0]) > 0.1
        keep[8:] = True                                     # keep every constraint row
        w = rng.uniform(0.5, 2.0, A.shape[0])
        Ak = (sp.diags(w * keep) @ A).tocsr()
        xs = _exact(Ak, w * keep * b)
        with LSQSolver(0) as s:
            Ac = A.tocoo()
            s.set_matrix_coo(Ac.shape[0], Ac.shape[1], Ac.row, Ac.col, Ac.data)
            x0, _ = s.solve(b, atol=1e-12, btol=1e-12, precond=5)          # factor for unit weights
            s.set_row_weight(w)
            s.set_row_mask(keep)
            x, st = s.solve(b, atol=1e-12, btol=1e-12, precond=5)          # must refactor
        assert st['istop'] in (1, 2) and st['iters'] <= 30, (nodes, st)
        assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8, nodes


def test_precond5_rank_deficient_raises(gpu_available):
    from lssurf_amd._native import NativeError
    A = sp.coo_matrix(np.array([[1.0, 1.0, 0.0], [2.0, 2.0, 0.0], [0.0, 0.0, 1.0]]))   # columns 0, 1 equal
    with LSQSolver(0) as s:
        s.set_matrix_coo(3, 3, A.row, A.col, A.data)
        with pytest.raises(NativeError):
            s.solve(np.ones(3), precond=5)
