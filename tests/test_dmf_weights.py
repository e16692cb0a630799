"""Host restatement of the CGNR matrix-free data rows (lsqr_cg.inc k_cg_dmf_ad / k_cg_dmf_atq,
assemble.hip build_dmf): a data row is rebuilt from its point's float subscripts
f_d = (p_d - b0_d) / delta_d alone — cell = floor(f) clamped to the last cell, fraction
f - cell, weights w = ((1*a_y)*a_x)*a_t — and must reproduce the interpolation rows of the host
lin_op (lin_op.interp_mtx, reference lin_op.py:163-247) bit for bit: same columns, same values.
Also pins the (y, x)-cell counting sort: every node's Ad^T gather over its <= 4 cells visits
exactly the points whose rows hold that node.  CPU only."""
import numpy as np
import scipy.sparse as sp

import lssurf_amd as LS
from lssurf_amd import assemble, synthetic


def _cell(f, n):
    c = np.floor(f)
    fr = f - c
    c = c.astype(np.int64)
    over = (c > n - 2) | (c < 0)
    c = np.clip(c, 0, n - 2)
    fr = np.where(over, f - c, fr)
    return c, fr


def _dmf_rows(gdesc, interp, coords):
    """(rows, cols, vals) of the data rows as k_cg_dmf_ad forms them (row scale 1)."""
    g0 = gdesc[interp[0]]
    py, px = coords[0], coords[1]
    fy = (py - g0.b0[0]) / g0.delta[0]
    fx = (px - g0.b0[1]) / g0.delta[1]
    S0, S1 = int(g0.shape[0]), int(g0.shape[1])
    cy, ry = _cell(fy, S0)
    cx, rx = _cell(fx, S1)
    ay, ax = 1.0 - ry, 1.0 - rx
    w2 = {(0, 0): ay * ax, (0, 1): ay * rx, (1, 0): ry * ax, (1, 1): ry * rx}
    R, C, V = [], [], []
    n = py.size
    for k in interp:
        g = gdesc[k]
        if g.ndim == 2:
            for (by, bx), w in w2.items():
                R.append(np.arange(n)); C.append(g.col0 + (cy + by) * S1 + cx + bx); V.append(w)
        else:
            S2 = int(g.shape[2])
            ft = (coords[2] - g.b0[2]) / g.delta[2]
            ct, rt = _cell(ft, S2)
            for (by, bx), w in w2.items():
                for bt, a in ((0, 1.0 - rt), (1, rt)):
                    R.append(np.arange(n))
                    C.append(g.col0 + ((cy + by) * S1 + cx + bx) * S2 + ct + bt)
                    V.append(w * a)
    return np.concatenate(R), np.concatenate(C), np.concatenate(V), (cy, cx, S0, S1)


def _system(name):
    D, kw = synthetic.points(name)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    gdesc, interp, coords, stencils, npts = assemble.describe(S['G_data'], S['Gc'])
    return S, gdesc, list(interp), coords, npts


def test_matrix_free_rows_equal_lin_op_rows():
    for name in ('t64', 't15'):
        S, gdesc, interp, coords, npts = _system(name)
        r, c, v, _ = _dmf_rows(gdesc, interp, coords)
        n_full = int(S['G_data'].col_N)
        Gm = sp.coo_matrix((v, (r, c)), shape=(npts, n_full)).tocsr()
        Gm.eliminate_zeros()
        Gh = S['G_data'].toCSR()[:npts].tocsr()
        Gh.eliminate_zeros()
        Gm.sort_indices(); Gh.sort_indices()
        assert np.array_equal(Gm.indptr, Gh.indptr) and np.array_equal(Gm.indices, Gh.indices), name
        assert np.array_equal(Gm.data, Gh.data), name       # bit-identical weights


def test_points_on_the_upper_bound_keep_their_weights():
    """f = S - 1 exactly: the last cell with fraction 1 gives the node weight 1 as lin_op's
    (cell S - 1, fraction 0) row does."""
    f = np.array([0.0, 0.25, 62.5, 63.0])
    c, fr = _cell(f, 64)
    assert list(c) == [0, 0, 62, 62] and list(fr) == [0.0, 0.25, 0.5, 1.0]


def test_cell_sorted_gather_visits_every_row_of_a_node():
    S, gdesc, interp, coords, npts = _system('tdense')
    r, c, v, (cy, cx, S0, S1) = _dmf_rows(gdesc, interp, coords)
    key = cy * (S1 - 1) + cx
    order = np.argsort(key, kind='stable')                 # build_dmf's counting sort
    ptr = np.zeros((S0 - 1) * (S1 - 1) + 1, np.int64)
    np.add.at(ptr, key + 1, 1)
    ptr = np.cumsum(ptr)
    z0 = gdesc[interp[0]]
    rng = np.random.default_rng(1)
    for node in rng.integers(0, S0 * S1, 200):
        iy, ix = divmod(int(node), S1)
        seen = []
        for yy in (iy - 1, iy):                             # cell rows of the node
            if 0 <= yy <= S0 - 2:
                lo, hi = max(ix - 1, 0), min(ix, S1 - 2)
                seen.extend(order[ptr[yy * (S1 - 1) + lo]:ptr[yy * (S1 - 1) + hi + 1]].tolist())
        col = z0.col0 + node
        rows = np.unique(r[(c == col) & (v != 0)])
        assert set(rows.tolist()) <= set(seen), node
