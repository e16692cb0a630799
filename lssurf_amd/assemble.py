"""Structured (device-side) formation of the smooth_fit operator.

Turns the structure that lin_op records (``parts``: interpolation of points into fd_grids,
constant-coefficient stencils over the valid centres of a grid) into the descriptors of
``lsq_set_matrix_stencil`` (include/lsqsurf.h), so the device generates every row itself —
no host triplets, no PCIe transfer of the 24 B/entry COO.  Returns None for operators whose
values were changed by data (masks, normalisation, biases), which then go through the COO
path.

Field-valued parts (``describe(..., with_fields=True)``): stencil parts whose rows were scaled
row by row (lin_op.scale_rows — the anisotropic notebook's directional operator, cells 9-10) or
that share their rows with other stencil parts (lin_op.add) become ONE part per row set with the
union of their offsets and exact per-row values, handed to ``lsq_set_stencil_fields``: the
values of offset t summed over the parts in part order (what scipy's duplicate summation in
lin_op.toCSR computes; exact for the ≤ 2 nonzero terms per entry of the directional operator),
stored as distinct fields F_j with entry t = ±F_{fsel_t}.
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


def _part_values(p):
    """(n_eq,) value array (or a scalar) of every template entry of stencil part p after its
    value chain — v[:, t] = vals[t], then each chain step in order (lin_op.scale_rows /
    scale_values), exactly as the reference's in-place products."""
    out = []
    for t in range(len(p['vals'])):
        v = p['vals'][t]
        for kind, s in p.get('chain', []):
            v = v * s
        out.append(v)
    return out


def _merge_group(group, n_eq):
    """One field-valued part from stencil parts on the same rows: (offsets, val, fsel, F)."""
    offs, vals = [], []
    for p in group:
        nd = len(p['subs'])
        for t, v in enumerate(_part_values(p)):
            o = tuple(int(p['subs'][d][t]) for d in range(nd)) + (0,) * (3 - nd)
            arr = np.broadcast_to(np.asarray(v, dtype=float), (n_eq,))
            if o in offs:
                k = offs.index(o)
                vals[k] = vals[k] + arr          # duplicate (row, col): summed in part order
            else:
                offs.append(o)
                vals.append(np.array(arr))
    fields, fsel, sign = [], [], []
    for v in vals:
        for j, f in enumerate(fields):
            if np.array_equal(v, f):
                fsel.append(j)
                sign.append(1.0)
                break
            if np.array_equal(v, -f):
                fsel.append(j)
                sign.append(-1.0)
                break
        else:
            fsel.append(len(fields))
            sign.append(1.0)
            fields.append(v)
    return (np.asarray(offs, dtype=np.int32), np.asarray(sign), np.asarray(fsel, dtype=np.int32),
            np.ascontiguousarray(np.stack(fields)))


def describe(G_data, Gc, with_fields=False):
    """(grids, interp_grid_ids, (py, px, pt), stencils, npts) or None if not structured;
    with_fields: a sixth element, the field-valued parts [(stencil index, off, val, fsel, F)]
    (None is returned for such operators when with_fields is False)."""
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
    # stencil parts, grouped by row set (parts added onto the same rows are consecutive)
    groups = []
    for p in Gc.parts:
        if p['kind'] != 'stencil' or p.get('row_base', 0) != 0:
            return None
        key = (id(p['grid']), int(p['row0']), int(p['n_eq']), tuple(p['lo']), tuple(p['hi']))
        if groups and groups[-1][0] == key:
            groups[-1][1].append(p)
        else:
            if any(g[0][1] == key[1] and g[0][2] for g in groups):
                return None   # a row set split by other parts: not a tiling of the rows
            groups.append((key, [p]))
    stencils, fields = [], []
    for key, group in groups:
        p = group[0]
        s = StencilDesc()
        s.grid = gid(p['grid'])
        nd = len(p['subs'])
        s.row0 = npts + int(p['row0'])
        s.n_eq = int(p['n_eq'])
        for d in range(nd):
            s.lo[d] = int(p['lo'][d])
            s.hi[d] = int(p['hi'][d])
        plain = len(group) == 1 and not p.get('chain')
        if plain:
            if len(p['vals']) > 8:
                return None
            s.ntpl = len(p['vals'])
            for t in range(s.ntpl):
                for d in range(nd):
                    s.off[t][d] = int(p['subs'][d][t])
                s.val[t] = float(p['vals'][t])
        else:
            if not with_fields:
                return None
            off, val, fsel, F = _merge_group(group, s.n_eq)
            if off.shape[0] > 16:
                return None
            s.ntpl = 1          # replaced by lsq_set_stencil_fields
            s.val[0] = 1.0
            fields.append((len(stencils), off, val, fsel, F))
        stencils.append(s)
    if len(grids) > 4 or len(stencils) > 32:
        return None
    py = np.ascontiguousarray(coords[0], dtype=np.float64)
    px = np.ascontiguousarray(coords[1], dtype=np.float64)
    pt = np.ascontiguousarray(coords[2], dtype=np.float64) if len(coords) > 2 else None
    out = [_grid_desc(g) for g in grids], interp, (py, px, pt), stencils, npts
    return out + (fields,) if with_fields else out
