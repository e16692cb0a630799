"""GPU triangular kernels vs the reference Cython kernels (golden I/O, bit-for-bit) and vs the
oracle's C restatement on larger random factors."""
import numpy as np
import pytest
import scipy.sparse as sp

import lssurf_amd as LS
from conftest import golden, golden_csr
from oracle import cpu

pytestmark = pytest.mark.gpu


def _cases():
    d = golden('tri.npz')
    for i in range(int(d['ncases'])):
        yield i, d, golden_csr(d, f'R{i}')


def test_inv_tr_upper_bitwise(gpu_available):
    for i, d, R in _cases():
        for tag in ('inv', 'ovf'):
            rr, cc, vv, st = LS.inv_tr_upper(R, int(d[f'{tag}{i}_nnz']), 1e-5)
            assert st == int(d[f'{tag}{i}_st']), (i, tag)
            np.testing.assert_array_equal(rr, d[f'{tag}{i}_rr'])
            np.testing.assert_array_equal(cc, d[f'{tag}{i}_cc'])
            np.testing.assert_array_equal(vv, d[f'{tag}{i}_vv'])


def test_rowrss_and_solve_bitwise(gpu_available):
    for i, d, R in _cases():
        np.testing.assert_array_equal(LS.propagate_qz_errors(R), d[f'rss{i}'])
        np.testing.assert_array_equal(LS.spsolve_tr_upper(R, d[f'b{i}']), d[f'sol{i}'])


def _rand_R(rng, N, dens):
    R = sp.triu(sp.random(N, N, density=dens, random_state=rng), k=1).tocsr() + \
        sp.diags(rng.uniform(0.5, 2.0, N) * np.sign(rng.normal(size=N)))
    R = sp.csr_matrix(R)
    R.sort_indices()
    return R


@pytest.mark.parametrize('N,dens', [(300, 0.03), (700, 0.01)])
def test_tri_vs_oracle_random(gpu_available, N, dens):
    rng = np.random.default_rng(N)
    R = _rand_R(rng, N, dens)
    for nnz in (N * N, N * 3):   # roomy buffer and an overflowing one
        a = LS.inv_tr_upper(R, nnz, 1e-5)
        b = cpu.inv_tr_upper(R, nnz, 1e-5)
        assert a[3] == b[3]
        for x, y in zip(a[:3], b[:3]):
            np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(LS.propagate_qz_errors(R), cpu.propagate_qz_errors(R))
    bb = rng.normal(size=N)
    np.testing.assert_array_equal(LS.spsolve_tr_upper(R, bb), cpu.spsolve_tr_upper(R, bb))


def test_rss_is_diag_of_inverse(gpu_available):
    rng = np.random.default_rng(2)
    R = _rand_R(rng, 150, 0.05)
    Rinv = np.linalg.inv(R.toarray())
    np.testing.assert_allclose(LS.propagate_qz_errors(R), np.sqrt((Rinv ** 2).sum(axis=1)), rtol=1e-12)
