"""Structured (device-side) formation of the smooth_fit operator.

Turns the structure that lin_op records (``parts``: interpolation of points into fd_grids,
constant-coefficient stencils over the valid centres of a grid) into the descriptors of
``lsq_set_matrix_stencil`` (include/lsqsurf.h), so the device generates every row itself —
no host triplets, no PCIe transfer of the 24 B/entry COO.  Returns None for operators whose
values were changed by data (masks, normalisation, biases), which then go through the COO
path.
"""
import numpy as np

from ._native import GridDesc, StencilDesc


def _grid_desc(g):
    d = GridDesc()
    d.ndim = int(g.N_dims)
    for k in range(d.ndim):
        d.shape[k] = int(g.shape[k])
        d.b0[k] = float(g.bds[k][0])
        d.delta[k] = float(g.delta[k])
    d.col0 = int(g.col_0)
    return d


def describe(G_data, Gc):
    """(grids, interp_grid_ids, (py, px, pt), stencils, npts) or None if not structured."""
    if G_data.parts is None or Gc.parts is None or not G_data.parts:
        return None
    grids, index = [], {}

    def gid(g):
        if id(g) not in index:
            index[id(g)] = len(grids)
            grids.append(g)
        return index[id(g)]

    npts = int(G_data.N_eq)
    interp, coords = [], None
    for p in G_data.parts:
        if p['kind'] != 'interp' or p['n_eq'] != npts or p['rows'].size != npts or \
                not np.array_equal(p['rows'], np.arange(npts)):
            return None
        interp.append(gid(p['grid']))
        pts = p['pts']
        if coords is None or len(pts) > len(coords):
            if coords is not None and any(not np.array_equal(a, b) for a, b in zip(coords, pts)):
                return None
            coords = pts
    stencils = []
    for p in Gc.parts:
        if p['kind'] != 'stencil' or p.get('row_base', 0) != 0 or len(p['vals']) > 8:
            return None
        s = StencilDesc()
        s.grid = gid(p['grid'])
        s.ntpl = len(p['vals'])
        nd = len(p['subs'])
        for t in range(s.ntpl):
            for d in range(nd):
                s.off[t][d] = int(p['subs'][d][t])
            s.val[t] = float(p['vals'][t])
        s.row0 = npts + int(p['row0'])
        s.n_eq = int(p['n_eq'])
        for d in range(nd):
            s.lo[d] = int(p['lo'][d])
            s.hi[d] = int(p['hi'][d])
        stencils.append(s)
    if len(grids) > 4 or len(stencils) > 32:
        return None
    py = np.ascontiguousarray(coords[0], dtype=np.float64)
    px = np.ascontiguousarray(coords[1], dtype=np.float64)
    pt = np.ascontiguousarray(coords[2], dtype=np.float64) if len(coords) > 2 else None
    return [_grid_desc(g) for g in grids], interp, (py, px, pt), stencils, npts
