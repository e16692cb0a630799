"""Host logic of sparseqr_compat's band order (CPU): AᵀA bandwidth from A's row spans, and the
reverse Cuthill-McKee fallback for column orders that are not banded."""
import numpy as np
import scipy.sparse as sp

from lssurf_amd import aniso
from lssurf_amd import sparseqr_compat as sc


def test_ata_bandwidth_matches_formed_normal_matrix():
    A, b, g = aniso.system(31, npts=200)
    N = (sp.csr_matrix(A).T @ sp.csr_matrix(A)).tocoo()
    assert sc.ata_bandwidth(A) == int(np.abs(N.row - N.col).max())
    perm = np.random.default_rng(0).permutation(A.shape[1])
    pos = np.empty_like(perm)
    pos[perm] = np.arange(perm.size)
    assert sc.ata_bandwidth(A, perm) == int(np.abs(pos[N.row] - pos[N.col]).max())


def test_band_order_natural_and_rcm(monkeypatch):
    A, b, g = aniso.system(41, npts=300)
    perm, bw = sc.band_order(A)
    assert perm is None and bw <= 2 * 41 + 2              # 3×3 stencil: AᵀA reaches ±2 node rows
    shuffle = np.random.default_rng(3).permutation(A.shape[1])
    As = sp.csr_matrix(A)[:, shuffle]
    monkeypatch.setattr(sc, 'BAND_MAX_COLS', 200)
    perm, bw = sc.band_order(As)
    assert perm is not None and np.array_equal(np.sort(perm), np.arange(A.shape[1]))
    assert bw < sc.ata_bandwidth(As) / 5


def test_aniso_system_shape():
    A, b, g = aniso.system(21)
    n = 21 * 21
    assert A.shape[1] == n and A.shape[0] == 8 + 19 * 19 + n   # 8 points, Axy on interior nodes, mag on all
    assert np.all(np.isfinite(A.data)) and b.shape == (A.shape[0],)
