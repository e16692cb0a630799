"""GPU diagnostic (development): band vs dense error propagation against a host sparse LU of AᵀA
on the columns where they differ most.   python tools/band_debug.py 48"""
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0] + '/tools')
from bench_errors import system  # noqa: E402
from lssurf_amd.constraint_functions import reference_epoch_keep_cols  # noqa: E402
from lssurf_amd.errors import band_order  # noqa: E402
from lssurf_amd.smooth_fit import FitSystem  # noqa: E402


def main(S):
    o = system(S)
    keep = reference_epoch_keep_cols(o['G_data'].col_N, o['grids']['dz'], 6)
    fs = FitSystem(o['G_data'], o['Gc'], keep, o['Gc'].col_N, device=0)
    try:
        w = 1. / np.concatenate([o['Ed'], o['Ec']])
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.ones(fs.n_data + fs.n_con, bool))
        perm = band_order(o['grids'], keep)
        Eb, _, info = fs.solver.cov_band(perm)
        Eb_rev, _, _ = fs.solver.cov_band(perm[::-1].copy())
        Ed = fs.solver.sigma_x()
        A = fs.solver.get_csr()
    finally:
        fs.close()
    print('info', info.tolist(), flush=True)
    if len(sys.argv) > 2:        # save for a host-side analysis (the LU below is slow)
        A = A.tocsr()
        np.savez(sys.argv[2], Eb=Eb, Eb_rev=Eb_rev, Ed=Ed, indptr=A.indptr, indices=A.indices, data=A.data,
                 shape=np.array(A.shape))
        return
    Aw = A                       # lsq_get_csr: the weighted, masked operator
    N = (Aw.T @ Aw).tocsc()
    d = np.abs(Eb - Ed)
    worst = np.argsort(d)[-8:]
    rng = np.random.default_rng(0)
    cols = np.concatenate([worst, rng.choice(Eb.size, 8, replace=False)])
    lu = spla.splu(N, permc_spec='MMD_AT_PLUS_A')
    for c in cols:
        e = np.zeros(N.shape[0])
        e[c] = 1.0
        x = lu.solve(e)
        x = x + lu.solve(e - N @ x)          # one refinement step
        ex = np.sqrt(x[c])
        print(f'col {c:6d}  exact {ex:.12e}  band {abs(Eb[c] - ex) / ex:.2e}  band(rev) '
              f'{abs(Eb_rev[c] - ex) / ex:.2e}  dense {abs(Ed[c] - ex) / ex:.2e}')
    print('band vs dense max rel', d.max() / np.abs(Ed).max(), ' band vs band(rev)',
          np.abs(Eb - Eb_rev).max() / np.abs(Eb).max())


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 48)
