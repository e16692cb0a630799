"""Error propagation for smooth_fit(compute_E=True) — LSsurf/smooth_fit.py:212-274.

The reference factors A = Q R E' with ``sparseqr.rz`` (:218), inverts R column by column with
the Cython ``inv_tr_upper`` keeping |x| > 1e-5 (:240-248), and reports
``E0 = sqrt(row sums of Rinv²)`` (:253) mapped through Ip_c onto the z0 / dz grids, plus
``op.grid_error(Ip_c·Rinv)`` for the averaging operators (:266-270).  Mathematically
E0 = sqrt(diag((AᵀA)⁻¹)) for any R with RᵀR = AᵀA, so lssurf_amd forms AᵀA and its Cholesky
factor R on the device (liblsqsurf dense path) and computes the row RSS of R⁻¹ there, without
the 1e-5 drop tolerance (the reference's truncation changes E0 by ~sqrt(#dropped)·1e-5; see
DESIGN.md §Parity).
"""
from time import time

import numpy as np
import scipy.sparse as sp

from . import containers as pc
from .smooth_fit import FitSystem


def calc_and_parse_errors(E, G_data, Gc, Ed, Ec, data, in_TSE, keep_cols, grids, avg_ops, device=0, timing=None):
    timing = {} if timing is None else timing
    tic = time()
    sigma_data = np.sqrt(Ed ** 2 + data.sigma_extra ** 2)
    E_all = np.concatenate((sigma_data, Ec))
    w = 1. / E_all                                   # TCinv, smooth_fit.py:697
    fs = FitSystem(G_data, Gc, keep_cols, Gc.col_N, device=device)
    try:
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.concatenate([np.asarray(in_TSE, bool), np.ones(Gc.N_eq, bool)]))
        E0c = fs.solver.sigma_x()
        timing['decompose_qz'] = time() - tic
        Rinv = fs.solver.rinv() if avg_ops else None
    finally:
        fs.close()
    timing['propagate_errors'] = time() - tic
    E0 = np.zeros(Gc.col_N)
    E0[keep_cols] = E0c
    z0g, dzg = grids['z0'], grids['dz']
    E['sigma_z0'] = pc.grid.data().from_dict({'x': z0g.ctrs[1], 'y': z0g.ctrs[0],
                                              'sigma_z0': np.reshape(E0[Gc.TOC['cols']['z0']], z0g.shape)})
    E['sigma_dz'] = pc.grid.data().from_dict({'x': dzg.ctrs[1], 'y': dzg.ctrs[0], 'time': dzg.ctrs[2],
                                              'sigma_dz': np.reshape(E0[Gc.TOC['cols']['dz']], dzg.shape)})
    if avg_ops:
        full = np.zeros((Gc.col_N, Rinv.shape[1]))
        full[keep_cols] = Rinv                       # Ip_c · Rinv
        for key, op in avg_ops.items():
            fields = {coord: ctr for coord, ctr in zip(op.dst_grid.coords, op.dst_grid.ctrs)}
            fields['sigma_' + key] = op.grid_error(sp.csr_matrix(full))
            E['sigma_' + key] = pc.grid.data().from_dict(fields)
    return E
