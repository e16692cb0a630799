"""Error propagation for smooth_fit(compute_E=True) — LSsurf/smooth_fit.py:212-274.

The reference factors A = Q R E' with ``sparseqr.rz`` (:218), inverts R column by column with
the Cython ``inv_tr_upper`` keeping |x| > 1e-5 (:240-248), and reports
``E0 = sqrt(row sums of Rinv²)`` (:253) mapped through Ip_c onto the z0 / dz grids, plus
``op.grid_error(Ip_c·Rinv)`` for the averaging operators (:266-270).  Mathematically
E0 = sqrt(diag((AᵀA)⁻¹)) for any R with RᵀR = AᵀA, so lssurf_amd forms AᵀA and its Cholesky
factor R on the device (liblsqsurf dense path) and computes the row RSS of R⁻¹ there, without
the 1e-5 drop tolerance (the reference's truncation changes E0 by ~sqrt(#dropped)·1e-5; see
DESIGN.md §Parity).

Default (`method='band'`): no dense factor — the columns are ordered by node position
(`band_order`), AᵀA is factored inside its band and the rows of R⁻¹ are formed by banded forward
sweeps without being stored (liblsqsurf `lsq_cov_band`, csrc/band.hip); the averaging operators'
errors sqrt(diag(op (AᵀA)⁻¹ opᵀ)) come from sweeps with the op rows as right-hand sides.
`method='dense'` keeps the n × n factor and R⁻¹ (n ≲ 3·10⁴).

At scale (`method='window'`, and `'auto'` above WINDOW_MIN_COLS columns): the band of AᵀA grows
with the lattice width (O(n·w²) work, O(n·w) memory: infeasible past ~2·10⁵ columns).  (AᵀA)⁻¹'s
correlations decay with node distance (measured: |corr| 0.30 / 0.11 / 0.03 / 0.018 at 2 / 4 / 6 /
8 nodes, t64-type systems), so diag((AᵀA)⁻¹) of the nodes of a tile is that of the principal
submatrix over the tile plus a margin of nodes — the variance conditional on the columns outside
held fixed differs from the marginal one by the correlations across the margin.  Tiles of
`tile` × `tile` nodes of the (coarser) dz lattice, windows of ± `margin` nodes, each factored in
its band on the device (lsq_cov_band_window); the averaging operators' rows go with the tile of
their support's centre (their support must lie inside the window).  Accuracy against the full
band factor: DESIGN.md §Error propagation (tests/test_gpu_errors_window.py).
"""
import os
from time import time

import numpy as np
import scipy.sparse as sp

from . import containers as pc
from .smooth_fit import FitSystem
from ._native import NativeError


def band_order(grids, keep_cols):
    """New position -> compact column: columns ordered by node position (y, then x), then grid,
    then epoch, so that AᵀA of a smooth_fit system is banded (z0 and dz of a node adjacent, a band
    of ~2 node rows).  Columns outside every grid go last."""
    gl = [g for g in grids.values() if getattr(g, 'N_dims', 0) >= 2]
    n_full = max(int(g.col_N) for g in gl)
    key = np.full((4, n_full), np.inf)
    for gi, g in enumerate(gl):
        sub = np.unravel_index(np.arange(int(g.N_nodes)), tuple(g.shape))
        idx = np.arange(g.col_0, g.col_0 + int(g.N_nodes))
        key[0, idx] = g.ctrs[0][sub[0]]
        key[1, idx] = g.ctrs[1][sub[1]]
        key[2, idx] = gi
        key[3, idx] = sub[2] if g.N_dims > 2 else -1
    k = key[:, keep_cols]
    return np.lexsort((k[3], k[2], k[1], k[0])).astype(np.int32)


WINDOW_MIN_COLS = 250_000      # 'auto': the full band below, tiled windows above
# tile 32 (round 5; 64 before): a window's interior sweeps cost ~(margin + tile/2)·(tile + 2·margin)²
# per column, so 32-node tiles do 2.4× fewer tile products at C4 (4.2·10⁹ against 1.0·10¹⁰) for
# 4× the windows, whose factorizations now run beside other windows' sweeps; σ within 3.5e-6 of
# the full band at 256²×12 (64-node tiles: 1.7e-6), the same self-check at C4 (7.1e-7)
WINDOW_TILE, WINDOW_MARGIN = 32, 24
WINDOW_BATCH = 64              # windows per lsq_cov_band_windows call (host memory of their column lists)
WINDOW_CHECK_TOL = 1e-4        # self-check bound: σ of a sample tile at twice the margin (the margin
                               # doubles, up to 4×, until it holds; the reference's own Rinv
                               # truncation moves σ by ~1e-5)


def _node_index(grids, keep_cols):
    """(iy, ix, dy, dx) per compact column: node indices on the coarsest (y, x) lattice of the grids
    (a finer z0 node maps to the coarse cell it lies in) and that lattice's spacing."""
    gl = [g for g in grids.values() if getattr(g, 'N_dims', 0) >= 2]
    n_full = max(int(g.col_N) for g in gl)
    dy = max(float(g.delta[0]) for g in gl)
    dx = max(float(g.delta[1]) for g in gl)
    y0 = min(float(g.ctrs[0][0]) for g in gl)
    x0 = min(float(g.ctrs[1][0]) for g in gl)
    iy = np.zeros(n_full, np.int64)
    ix = np.zeros(n_full, np.int64)
    for g in gl:
        sub = np.unravel_index(np.arange(int(g.N_nodes)), tuple(g.shape))
        idx = np.arange(g.col_0, g.col_0 + int(g.N_nodes))
        iy[idx] = np.floor((g.ctrs[0][sub[0]] - y0) / dy + 1e-9).astype(np.int64)
        ix[idx] = np.floor((g.ctrs[1][sub[1]] - x0) / dx + 1e-9).astype(np.int64)
    return iy[keep_cols], ix[keep_cols]


SCHUR_DEPTH = 2   # node rows of the interior the bottom margin's rows reach (AᵀA couples ±2 rows)


def window_cov(solver, grids, keep_cols, op=None, tile=WINDOW_TILE, margin=WINDOW_MARGIN, timing=None, schur=None):
    """(E, op_err) of the current weighted, masked system by tiled windows (module docstring):
    E[c] ≈ sqrt(((AᵀA)⁻¹)_cc) per compact column, op_err[i] ≈ sqrt(op_i (AᵀA)⁻¹ op_iᵀ).

    schur (default: on when there are no op rows; LSQ_E_SCHUR=0 turns it off): each window's bottom
    margin is eliminated first (lsq_cov_band_windows_schur) — the same conditional variance, with
    the sweeps ending at the interior instead of the window's end (DESIGN.md §Error propagation)."""
    iy, ix = _node_index(grids, keep_cols)
    order = band_order(grids, keep_cols)
    n = iy.size
    E = np.zeros(n)
    op_err = None
    ny, nx = int(iy.max()) + 1, int(ix.max()) + 1
    iy_o, ix_o = iy[order], ix[order]
    if op is not None:   # every op row with its support's node box; rows go with the tile of its centre
        op = sp.csr_matrix(op)
        op_err = np.zeros(op.shape[0])
        nr = op.shape[0]
        rows_of = np.repeat(np.arange(nr), np.diff(op.indptr))
        big = np.iinfo(np.int64).max
        y_lo = np.full(nr, big); y_hi = np.full(nr, -1); x_lo = np.full(nr, big); x_hi = np.full(nr, -1)
        np.minimum.at(y_lo, rows_of, iy[op.indices]); np.maximum.at(y_hi, rows_of, iy[op.indices])
        np.minimum.at(x_lo, rows_of, ix[op.indices]); np.maximum.at(x_hi, rows_of, ix[op.indices])
        empty = y_hi < 0
        y_lo[empty] = y_hi[empty] = x_lo[empty] = x_hi[empty] = 0
        oty, otx = (y_lo + y_hi) // 2 // tile, (x_lo + x_hi) // 2 // tile
        # rows whose support leaves their tile's window get windows of their own (support ± margin)
        own = (y_lo < oty * tile - margin) | (y_hi >= oty * tile + tile + margin) | \
              (x_lo < otx * tile - margin) | (x_hi >= otx * tile + tile + margin)

    # window positions without a pass over all n columns: the band order sorts by node row, so a
    # window's rows are one contiguous run of it, filtered by node column (round 5: the full-length
    # masks and the n-long E of every window were ~0.2 s of host work per window at C4)
    rows_sorted = bool(np.all(iy_o[1:] >= iy_o[:-1]))
    if schur is None:
        schur = op is None and os.environ.get('LSQ_E_SCHUR', '1') != '0'
    schur = bool(schur) and rows_sorted and op is None
    depth = SCHUR_DEPTH

    def window(y0, y1, x0, x1):   # band-order positions of the nodes [y0, y1) × [x0, x1)
        a, b = (np.searchsorted(iy_o, y0, 'left'), np.searchsorted(iy_o, y1, 'left')) if rows_sorted else (0, n)
        yy, xx = iy_o[a:b], ix_o[a:b]
        m = (xx >= x0) & (xx < x1)
        if not rows_sorted:
            m &= (yy >= y0) & (yy < y1)
        return a + np.flatnonzero(m)

    # every window (tile ± margin, the op rows of the tile's centre; op rows wider than that get a
    # window of their own; last, the self-check: the most central tile with twice the margin) as a
    # small spec; its positions are formed only when its batch goes to the device
    # (lsq_cov_band_windows), so host memory stays O(WINDOW_BATCH windows) whatever the grid
    def tile_win(ty, tx, mg):
        if schur:   # A = [top margin, interior] rows; B' = reverse([Ib, bottom margin] rows)
            yb = min(ty + tile, ny)
            pos = window(ty - mg, yb, tx - mg, tx + tile + mg)
            bot = window(yb - depth, ty + tile + mg, tx - mg, tx + tile + mg)[::-1] if yb < ny else None
            nib = int(np.count_nonzero(iy_o[pos] >= yb - depth))
            if bot is not None and (bot.size <= nib or nib == 0):
                bot = None
        else:
            pos = window(ty - mg, ty + tile + mg, tx - mg, tx + tile + mg)
            bot, nib = None, 0
        yi, xi = iy_o[pos], ix_o[pos]
        return pos, (yi >= ty) & (yi < ty + tile) & (xi >= tx) & (xi < tx + tile), bot, nib

    specs = [('tile', ty, tx) for ty in range(0, ny, tile) for tx in range(0, nx, tile)]
    ntiles = len(specs)
    if op is not None and own.any():   # one window per distinct support box
        boxes = np.stack([y_lo, y_hi, x_lo, x_hi], axis=1)
        for b in np.unique(boxes[own], axis=0):
            specs.append(('own', b, np.flatnonzero(own & np.all(boxes == b, axis=1))))
    nown = len(specs) - ntiles
    cy, cx = (ny // 2) // tile * tile, (nx // 2) // tile * tile
    m2 = 2 * margin
    specs.append(('check', cy, cx))

    def materialize(spec):   # (positions, inner flags or None, op rows or None, B' positions or None, nib)
        if spec[0] == 'tile':
            ty, tx = spec[1], spec[2]
            pos, inner, bot, nib = tile_win(ty, tx, margin)
            rows = None if op is None else np.flatnonzero((oty == ty // tile) & (otx == tx // tile) & ~own)
            return pos, inner, rows, bot, nib
        if spec[0] == 'own':
            b = spec[1]
            return window(b[0] - margin, b[1] + margin + 1, b[2] - margin, b[3] + margin + 1), None, spec[2], None, 0
        pos, inner, bot, nib = tile_win(spec[1], spec[2], m2)
        return pos, inner, None, bot, nib

    E2 = pos2 = inner2 = None
    wmax = products = 0
    t_all = time()
    batch = max(int(os.environ.get('LSQ_E_BATCH', WINDOW_BATCH)), 1)
    for c0 in range(0, len(specs), batch):
        chunk = [materialize(sp_) for sp_ in specs[c0:c0 + batch]]
        req = [(order[pos], inner if inner is not None else np.zeros(pos.size, bool),
                op[rows] if (op is not None and rows is not None and rows.size) else None)
               for pos, inner, rows, _, _ in chunk]
        if schur:
            while True:
                sreq = [(cols, inn, None if bot is None else order[bot], nib)
                        for (cols, inn, _), (_, _, _, bot, nib) in zip(req, chunk)]
                try:
                    Es, info = solver.cov_band_windows_schur(sreq)
                    break
                except NativeError as e:   # a row reaches further than Ib: split one node row deeper
                    if 'deeper Ib' not in str(e) or depth >= 2 * SCHUR_DEPTH:
                        raise
                    depth += 1
                    chunk = [materialize(sp_) for sp_ in specs[c0:c0 + batch]]
                    req = [(order[pos], inner if inner is not None else np.zeros(pos.size, bool), None)
                           for pos, inner, _, _, _ in chunk]
            oes = [None] * len(chunk)
        else:
            Es, oes, info = solver.cov_band_windows(req)
        wmax, products = max(wmax, int(info[0])), products + int(info[3])
        for k, ((pos, inner, rows, _, _), (cols, _, _), Et, oe) in enumerate(zip(chunk, req, Es, oes)):
            if c0 + k == len(specs) - 1:       # the self-check window
                E2, pos2, inner2 = Et, pos, inner
                continue
            if inner is not None:
                E[cols[inner]] = Et[inner]
            if oe is not None:
                op_err[rows] = oe
        del chunk, req, Es, oes
    # self-check: σ of the central tile's columns moves by the correlations the margin cut off
    # (conditional vs marginal variance)
    c2 = order[pos2][inner2]
    e1, e2 = E[c2], E2[inner2]
    sel = e2 > 0
    check = float(np.max(np.abs(e1[sel] - e2[sel]) / e2[sel])) if sel.any() else 0.0
    if timing is not None:
        timing['E_window'] = {'tiles': ntiles, 'op_windows': nown, 'tile': tile, 'margin': margin,
                              'max_band_tiles': wmax, 'tile_products': products, 'selfcheck_rel': check,
                              'selfcheck_margin': m2, 'time_s': time() - t_all, 'lanes': int(info[5]),
                              'batch': batch, 'schur': bool(schur), 'schur_depth': depth if schur else None}
    return E, op_err, check


def _compact_rows(op, keep_cols, n_full):
    """The op's CSR (rows = its output equations) over the compact columns: entries in removed
    columns dropped (Ip_c·Rinv has zero rows there, smooth_fit.py:266)."""
    rows = op.ind0 if op.dst_ind0 is None else op.dst_ind0
    A = op.toCSR(row_N=rows.size, col_N=n_full).tocsc()
    return A[:, keep_cols].tocsr()


def _grid_values(op, vals):
    """Place per-row values on the op's output grid (the layout of lin_op.grid_error)."""
    grid, rows = op._out_grid_and_rows(None)
    E = np.zeros(op.col_N) + np.nan
    E[rows] = vals
    return E[grid.col_0:grid.col_N].reshape(grid.shape)


def calc_and_parse_errors(E, G_data, Gc, Ed, Ec, data, in_TSE, keep_cols, grids, avg_ops, device=0, timing=None,
                          method='auto'):
    timing = {} if timing is None else timing
    tic = time()
    approx = None   # window method: how σ was approximated (attached to the output grids)
    sigma_data = np.sqrt(Ed ** 2 + data.sigma_extra ** 2)
    E_all = np.concatenate((sigma_data, Ec))
    w = 1. / E_all                                   # TCinv, smooth_fit.py:697
    fs = FitSystem(G_data, Gc, keep_cols, Gc.col_N, device=device)
    op_err = {}
    try:
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.concatenate([np.asarray(in_TSE, bool), np.ones(Gc.N_eq, bool)]))
        if method == 'auto':
            method = 'band' if keep_cols.size <= WINDOW_MIN_COLS else 'window'
        if method == 'window':
            keys = list(avg_ops)
            mats = [_compact_rows(avg_ops[k], keep_cols, Gc.col_N) for k in keys]
            op = sp.vstack(mats).tocsr() if mats else None
            # LSQ_E_TILE / LSQ_E_MARGIN: development overrides (A/B of the window geometry)
            tile = int(os.environ.get('LSQ_E_TILE', WINDOW_TILE))
            margin = m0 = int(os.environ.get('LSQ_E_MARGIN', WINDOW_MARGIN))
            while True:
                E0c, errs, check = window_cov(fs.solver, grids, keep_cols, op, tile=tile, margin=margin,
                                              timing=timing)
                if check <= WINDOW_CHECK_TOL or margin >= 4 * m0:
                    break
                print(f'calc_and_parse_errors: window sigma moved by {check:.1e} with twice the margin '
                      f'({margin} nodes); retrying with a margin of {2 * margin}', flush=True)
                margin *= 2
            if check > WINDOW_CHECK_TOL:
                print(f'calc_and_parse_errors: WARNING window sigma within {check:.1e} only (margin {margin} nodes)',
                      flush=True)
            approx = (f'window (conditional variance): tile {tile}, margin {margin} nodes, '
                      f'self-check {check:.1e} relative at twice the margin')
            timing['decompose_qz'] = time() - tic
            off = 0
            for k, m in zip(keys, mats):
                op_err[k] = errs[off:off + m.shape[0]]
                off += m.shape[0]
            Rinv = None
        elif method == 'band':
            keys = list(avg_ops)
            mats = [_compact_rows(avg_ops[k], keep_cols, Gc.col_N) for k in keys]
            op = sp.vstack(mats).tocsr() if mats else None
            E0c, errs, info = fs.solver.cov_band(band_order(grids, keep_cols), op)
            timing['decompose_qz'] = time() - tic
            timing['E_band'] = {'tiles': int(info[0]), 'tile_rows': int(info[1]), 'bytes': int(info[2]),
                                'tile_products': int(info[3])}
            off = 0
            for k, m in zip(keys, mats):
                op_err[k] = errs[off:off + m.shape[0]]
                off += m.shape[0]
            Rinv = None
        elif method == 'dense':
            E0c = fs.solver.sigma_x()
            timing['decompose_qz'] = time() - tic
            Rinv = fs.solver.rinv() if avg_ops else None
        else:
            raise ValueError(f'calc_and_parse_errors: unknown method {method!r}')
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
    if approx is not None:
        timing['E_approximate'] = approx
    if avg_ops:
        if Rinv is not None:
            full = np.zeros((Gc.col_N, Rinv.shape[1]))
            full[keep_cols] = Rinv                   # Ip_c · Rinv
            Rs = sp.csr_matrix(full)
        for key, op in avg_ops.items():
            fields = {coord: ctr for coord, ctr in zip(op.dst_grid.coords, op.dst_grid.ctrs)}
            fields['sigma_' + key] = op.grid_error(Rs) if Rinv is not None else _grid_values(op, op_err[key])
            E['sigma_' + key] = pc.grid.data().from_dict(fields)
    if approx is not None:   # every output grid says it is the windowed (conditional) variance
        for v in E.values():
            v.approximate = approx
    return E
