"""Host logic of the banded error propagation (lssurf_amd.errors.band_order): the node-major
column order makes AᵀA of a smooth_fit system banded (CPU; the factorisation itself is
tests/test_gpu_band.py)."""
import numpy as np
import scipy.sparse as sp

import lssurf_amd as LS
from lssurf_amd import synthetic
from lssurf_amd.constraint_functions import reference_epoch_keep_cols
from lssurf_amd.errors import band_order


def _system(S, nt, spacing_z0=100.):
    W = {'x': (S - 1) * 100., 'y': (S - 1) * 100., 't': (nt - 1) * 0.25}
    rng = np.random.default_rng(1)
    npts = 2 * S * S
    D = LS.containers.data().from_dict({'x': (rng.random(npts) - 0.5) * W['x'], 'y': (rng.random(npts) - 0.5) * W['y'],
                                        'time': (rng.random(npts) - 0.5) * W['t'], 'z': rng.normal(0, 1, npts),
                                        'sigma': np.full(npts, 0.1)})
    out = LS.smooth_fit(data=D, W=W, ctr={'x': 0., 'y': 0., 't': 0.},
                        spacing={'z0': spacing_z0, 'dz': 100., 'dt': 0.25},
                        E_RMS=dict(synthetic.E_RMS_NOTEBOOK), reference_epoch=nt // 2, return_fit_objects=True)
    keep = reference_epoch_keep_cols(out['G_data'].col_N, out['grids']['dz'], nt // 2)
    rows, cols, vals = [], [], []
    r0 = 0
    for op in (out['G_data'], out['Gc']):
        r, c, v = op.triplets()
        rows.append(r + r0)
        cols.append(c)
        vals.append(v)
        r0 += op.N_eq
    A = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(r0, out['Gc'].col_N))[:, keep]
    return out, keep, A


def _bandwidth(A, perm):
    pos = np.empty(perm.size, int)
    pos[perm] = np.arange(perm.size)
    N = (A.T @ A).tocoo()
    return int(np.abs(pos[N.row] - pos[N.col]).max())


def test_band_order_is_a_permutation_and_banded():
    S, nt = 20, 8
    out, keep, A = _system(S, nt)
    perm = band_order(out['grids'], keep)
    assert np.array_equal(np.sort(perm), np.arange(keep.size))
    b = _bandwidth(A, perm)
    per_node = nt                               # z0 + nt−1 kept epochs
    assert b <= (2 * S + 3) * per_node, b       # ≤ ~2 node rows (second differences reach ±2 rows... in y)
    assert b < _bandwidth(A, np.arange(keep.size)) / 5
    # node-major: the first node's z0 column comes first, then its kept dz epochs
    z0c = out['G_data'].TOC['cols']['z0']
    assert keep[perm[0]] == z0c[0]


def test_band_order_mixed_spacing():
    """z0 on a finer lattice than dz: the order still follows node position (y, then x)."""
    out, keep, A = _system(12, 4, spacing_z0=50.)
    perm = band_order(out['grids'], keep)
    assert np.array_equal(np.sort(perm), np.arange(keep.size))
    assert _bandwidth(A, perm) < _bandwidth(A, np.arange(keep.size)) / 2
