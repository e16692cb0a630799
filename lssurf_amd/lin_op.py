"""Sparse linear operators on fd_grid nodes (COO triplets + table of contents).

Host mirror of LSsurf/lin_op.py:12-753.  Every method that the solve path uses reproduces the
reference's triplets (r, c, v), ``ind0`` and TOC exactly, in the same order and with
bit-identical coefficients:

  diff_op        lin_op.py:80-132   constant-coefficient template at every centre whose
                                    template fits in the grid (meshgrid 'ij' order)
  one/grad/grad2/grad_dzdt/grad2_dzdt/d2z_dt2/dzdt/diff   lin_op.py:249-309 (stencil table below)
  interp_mtx     lin_op.py:163-247  bi/trilinear weights into the 2^N surrounding nodes
  add / vstack   lin_op.py:134-161, 555-631
  toCSR          lin_op.py:745-753  (drop exact zeros, sum duplicates)
  mask_for_ind0, normalize_by_unit_product, grid_prod, grid_error, update_dst_grid
  sum_to_grid3, apply_mask, apply_2d_mask, mean_of_mask   lin_op.py:347-488, 669-732 (averaging)

In addition each operator records its *structure* (``parts``): which stencil or interpolation
generated which rows.  lssurf_amd's device path uses it to know an operator is a pure
stencil/interp operator; methods that rescale values by data (normalize_by_unit_product,
masks) drop the structure.
"""
import weakref

import numpy as np
import scipy.sparse as sp

from .fd_grid import fd_grid

# Stencil table: (name suffix, per-dimension offsets, coefficient numerator array, denominator
# expression) — the denominators are evaluated with the reference's exact operation order.


def _grad_parts(g, DOF):
    c = np.array([-1., 1.]) / (g.delta[0])
    return [('d' + DOF + '_dx', ([0, 0], [-1, 0]), c),
            ('d' + DOF + '_dy', ([-1, 0], [0, 0]), c)]


def _grad2_parts(g, DOF):
    c = np.array([-1., 2., -1.]) / (g.delta[0] ** 2)
    cxy = 0.5 * np.array([-1., 1., 1., -1]) / (g.delta[0] ** 2)
    return [('d2' + DOF + '_dx2', ([0, 0, 0], [-1, 0, 1]), c),
            ('d2' + DOF + '_dy2', ([-1, 0, 1], [0, 0, 0]), c),
            ('d2' + DOF + '_dxdy', ([-1, -1, 1, 1], [-1, 1, -1, 1]), cxy)]


def _grad_dzdt_parts(g, DOF, t):
    c = np.array([-1., 1., 1., -1.]) / (t * g.delta[0] * g.delta[2])
    return [('d2' + DOF + '_dxdt', ([0, 0, 0, 0], [-1, 0, -1, 0], [-t, -t, 0, 0]), c),
            ('d2' + DOF + '_dydt', ([-1, 0, -1, 0], [0, 0, 0, 0], [-t, -t, 0, 0]), c)]


def _grad2_dzdt_parts(g, DOF, t):
    c = np.array([-1., 2., -1., 1., -2., 1.]) / (t * g.delta[0] ** 2. * g.delta[2])
    cxy = np.array([-1., 1., 1., -1., 1., -1., -1., 1.]) / (g.delta[0] ** 2 * g.delta[2])
    return [('d3' + DOF + '_dx2dt', ([0, 0, 0, 0, 0, 0], [-1, 0, 1, -1, 0, 1], [-t, -t, -t, 0, 0, 0]), c),
            ('d3' + DOF + '_dy2dt', ([-1, 0, 1, -1, 0, 1], [0, 0, 0, 0, 0, 0], [-t, -t, -t, 0, 0, 0]), c),
            ('d3' + DOF + '_dxdydt', ([-1, 0, -1, 0, -1, 0, -1, 0], [-1, -1, 0, 0, -1, -1, 0, 0],
                                      [-t, -t, -t, -t, 0, 0, 0, 0]), cxy)]


_RANGES = {}   # id(array) -> (weakref, first, last): TOC arrays this module made with _arange


def _arange(lo, hi, dtype=int):
    """np.arange(lo, hi), remembered as a contiguous range (TOC rows / cols of 10⁷–10⁸ entries:
    consumers then slice instead of scanning or fancy-indexing them)."""
    a = np.arange(lo, hi, dtype=dtype)
    if a.size:
        key = id(a)
        _RANGES[key] = (weakref.ref(a, lambda _r, k=key: _RANGES.pop(k, None)), int(lo), int(hi) - 1)
    return a


class TocRows(dict):
    """A lin_op's TOC['rows'] (equation name → row indices).  Contiguous runs — every TOC the
    mirror builds for smooth_fit's stacks, up to 73 M rows at C4 — are kept as (first, last) and
    materialised as np.arange (remembered by known_range) only when an entry is read; range_of
    gives the run without materialising it.  Reading an entry returns the reference's int array."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._rng = {}

    def set_range(self, key, lo, hi):
        """rows lo … hi − 1"""
        dict.__setitem__(self, key, None)
        self._rng[key] = (int(lo), int(hi) - 1)

    def range_of(self, key):
        if key in self._rng:
            return self._rng[key]
        return known_range(dict.__getitem__(self, key))

    def __getitem__(self, key):
        v = dict.__getitem__(self, key)
        if v is None and key in self._rng:
            lo, hi = self._rng[key]
            v = _arange(lo, hi + 1)
            dict.__setitem__(self, key, v)
        return v

    def __setitem__(self, key, v):
        self._rng.pop(key, None)
        dict.__setitem__(self, key, v)

    def get(self, key, default=None):
        return self[key] if key in self else default

    def items(self):
        return [(k, self[k]) for k in self]

    def values(self):
        return [self[k] for k in self]

    def copy(self):
        c = TocRows(dict.items(self))
        c._rng = dict(self._rng)
        return c


def toc_range(toc, key):
    """(first, last) of toc[key] when it is one contiguous run, without materialising it."""
    return toc.range_of(key) if isinstance(toc, TocRows) else known_range(toc[key])


def known_range(a):
    """(first, last) of an array made by _arange (and not since replaced), else None."""
    e = _RANGES.get(id(a))
    return (e[1], e[2]) if e is not None and e[0]() is a else None


def _as_range(a):
    """(first, last) when `a` is a contiguous ascending integer range, else None."""
    kr = known_range(a)
    if kr is not None:
        return kr
    a = np.asarray(a)
    if a.ndim != 1 or a.size == 0 or a.dtype.kind not in 'iu':
        return None
    lo, hi = int(a[0]), int(a[-1])
    if hi - lo + 1 != a.size:
        return None
    return (lo, hi) if np.array_equal(a, np.arange(lo, hi + 1, dtype=a.dtype)) else None


def _union_sorted(arrays):
    """np.unique(np.concatenate(arrays)) — computed from the index ranges when every array is a
    contiguous range (the TOC column sets of grid operators), which avoids sorting ~10⁷ entries."""
    if not arrays:
        return np.array([], int)
    seen, uniq = set(), []
    for a in arrays:                     # the grid operators share their column array (_grid_cols)
        if id(a) not in seen:
            seen.add(id(a))
            uniq.append(a)
    arrays = uniq
    ranges = [_as_range(a) for a in arrays]
    if any(r is None for r in ranges):
        return np.unique(np.concatenate(arrays))
    ranges.sort()
    merged = [list(ranges[0])]
    for lo, hi in ranges[1:]:
        if lo <= merged[-1][1] + 1:
            merged[-1][1] = max(merged[-1][1], hi)
        else:
            merged.append([lo, hi])
    dtype = np.result_type(*[np.asarray(a).dtype for a in arrays])
    if len(merged) == 1:
        return _arange(merged[0][0], merged[0][1] + 1, dtype=dtype)
    return np.concatenate([np.arange(lo, hi + 1, dtype=dtype) for lo, hi in merged])


def _grid_cols(g):
    """The column range of grid g as one shared array per grid (TOC 'cols'; read-only use)."""
    key = (g.col_0, g.N_nodes)
    cached = getattr(g, '_toc_cols', None)
    if cached is None or cached[0] != key:
        cached = (key, _arange(g.col_0, g.col_0 + g.N_nodes))
        g._toc_cols = cached
    return cached[1]


class lin_op:
    def __init__(self, grid=None, row_0=0, col_N=None, col_0=None, name=None):
        self.grid = grid
        self.col_0 = col_0 if col_0 is not None else (grid.col_0 if grid is not None else None)
        self.col_N = col_N if col_N is not None else (grid.col_N if grid is not None else None)
        self.row_0 = row_0
        self.N_eq = 0
        self.name = name
        self.id = None
        self._r = np.array([], dtype=int)
        self._c = np.array([], dtype=int)
        self._v = np.array([], dtype=float)
        self._ind0 = np.zeros([0], dtype=int)
        self._lazy = None         # callable -> (r, c, v, ind0), evaluated on first access
        self.TOC = {'rows': {}, 'cols': {}}
        self.dst_grid = None
        self.dst_ind0 = None
        self.expected = None
        self.prior = None
        self.shape = None
        self.size = None
        self.parts = []   # structure records (see module docstring)

    def __update_size_and_shape__(self):
        self.shape = (self.N_eq, self.col_N)

    # ---- lazy triplets: structure-only operators materialise (r, c, v, ind0) on first use -----
    def _materialize(self):
        if self._lazy is not None:
            f, self._lazy = self._lazy, None
            self._r, self._c, self._v, self._ind0 = f()

    def _prop(name, structural):
        def get(self):
            self._materialize()
            return getattr(self, '_' + name)

        def put(self, value):
            self._materialize()
            setattr(self, '_' + name, value)
            if structural:
                self.parts = None      # values changed from outside: structure no longer describes them
        return property(get, put)

    r = _prop('r', True)
    c = _prop('c', True)
    v = _prop('v', True)
    ind0 = _prop('ind0', False)
    del _prop

    @property
    def materialized(self):
        return self._lazy is None

    # ---- helpers ---------------------------------------------------------------------------
    def apply_xform(self, pts, xform=None, dims=(0, 1)):
        if xform is None:
            xform = self.grid.xform
        if xform is None:
            return pts
        P = np.c_[[np.ravel(p) for p in pts[0:len(xform['origin'])]]].T
        T = (P - xform['origin']) @ xform['basis_vectors']
        return [T[:, d].ravel() for d in dims]

    def ravel(self):
        if self._lazy is not None:
            f = self._lazy
            self._lazy = lambda: tuple(np.ravel(a) for a in f())
        else:
            self._r, self._c, self._v = np.ravel(self._r), np.ravel(self._c), np.ravel(self._v)
        return self

    def fix_dtypes(self):
        self._materialize()
        self._r = self._r.astype(int)
        self._c = self._c.astype(int)

    # ---- stencils ----------------------------------------------------------------------------
    def diff_op(self, delta_subs, vals, which_nodes=None, valid_equations_only=True):
        g = self.grid
        nd = min(len(delta_subs), g.N_dims)   # extra offset rows are ignored (zip semantics)
        lo = [max(0, -int(np.min(ds))) if valid_equations_only else 0 for ds in delta_subs[:nd]]
        hi = [min(int(g.shape[k]), int(g.shape[k]) - int(np.max(delta_subs[k])))
              if valid_equations_only else int(g.shape[k]) for k in range(nd)]
        n_tpl = len(delta_subs[0])
        row_0 = self.row_0

        def centres_of():
            cs = [s.ravel() for s in np.meshgrid(*[np.arange(a, b) for a, b in zip(lo, hi)], indexing='ij')]
            if which_nodes is not None:
                keep = np.isin(g.global_ind(cs), which_nodes)
                cs = [s[keep] for s in cs]
            return cs

        def build():
            cs = centres_of()
            n_eq = cs[0].size
            R = np.empty((n_eq, n_tpl), dtype=int)
            C = np.empty((n_eq, n_tpl), dtype=int)
            V = np.empty((n_eq, n_tpl), dtype=float)
            rows = row_0 + np.arange(0, n_eq, dtype=int)
            for k in range(n_tpl):
                sub = [cs[d] + delta_subs[d][k] for d in range(nd)]
                R[:, k] = rows
                if valid_equations_only:
                    C[:, k] = g.global_ind(sub)
                    V[:, k] = np.ravel(vals[k])
                else:
                    C[:, k], ok = g.global_ind(sub, return_valid=True)
                    V[:, k] = np.ravel(vals[k]) * np.ravel(ok)
            return R, C, V, g.global_ind(cs).ravel()

        simple = valid_equations_only and which_nodes is None and all(np.size(vv) == 1 for vv in vals)
        if simple:
            n_eq = int(np.prod([max(b - a, 0) for a, b in zip(lo, hi)]))
            self._lazy = build
            self.parts = [dict(kind='stencil', grid=g, subs=[list(map(int, ds)) for ds in delta_subs[:nd]],
                               vals=np.array([float(np.ravel(vals[k])[0]) for k in range(n_tpl)]),
                               lo=lo, hi=hi, row0=0, n_eq=n_eq, row_base=row_0)]
        else:
            self._lazy = None
            self._r, self._c, self._v, self._ind0 = build()
            n_eq = self._r.shape[0]
            self.parts = None
        self.N_eq = n_eq
        self.TOC['rows'] = TocRows()
        self.TOC['rows'].set_range(self.name, 0, self.N_eq)
        self.TOC['cols'] = {g.name: _grid_cols(g)}
        self.__update_size_and_shape__()
        return self

    def scale_rows(self, f):
        """v[:, col] *= f for every template column (per-row scale of a stencil operator; what
        notebooks/smooth_fit_demo_aniso.ipynb cell 9 does with the interpolated direction field).
        Stencil parts keep their structure: the scale joins the part's value chain."""
        f = np.asarray(f, dtype=float).ravel()
        return self._chain(('rows', f), lambda V: V * f[:, None] if V.ndim > 1 else V * f)

    def scale_values(self, c):
        """v *= c (a scalar; notebook cell 10's ``temp.v *= 2``), keeping the stencil structure."""
        c = float(c)
        return self._chain(('const', c), lambda V: V * c)

    def _chain(self, step, apply):
        if self.parts is not None and all(p['kind'] == 'stencil' and p['row0'] == 0 and p['n_eq'] == self.N_eq
                                          for p in self.parts):
            f = self._lazy if self._lazy is not None else (lambda a=(self._r, self._c, self._v, self._ind0): a)

            def build(f=f):
                r, c, v, i0 = f()
                return r, c, apply(v), i0
            self._lazy = build
            self.parts = [dict(p, chain=list(p.get('chain', [])) + [step]) for p in self.parts]
        else:
            self._materialize()
            self._v = apply(self._v)
            self.parts = None
        return self

    def _stack_named(self, parts):
        subops = [lin_op(self.grid, name=nm).diff_op(subs, coeffs) for nm, subs, coeffs in parts]
        return self.vstack(tuple(subops))

    def one(self, DOF='z', which_nodes=None):
        self.diff_op([[0]] * len(self.grid.shape), np.array([1.]), which_nodes=which_nodes)
        self.__update_size_and_shape__()
        return self

    def grad(self, DOF='z'):
        self._stack_named(_grad_parts(self.grid, DOF))
        self.__update_size_and_shape__()
        return self

    def grad2(self, DOF='z'):
        self._stack_named(_grad2_parts(self.grid, DOF))
        self.__update_size_and_shape__()
        return self

    def grad_dzdt(self, DOF='z', t_lag=1):
        self._stack_named(_grad_dzdt_parts(self.grid, DOF, t_lag))
        self.__update_size_and_shape__()
        return self

    def grad2_dzdt(self, DOF='z', t_lag=1):
        self._stack_named(_grad2_dzdt_parts(self.grid, DOF, t_lag))
        self.__update_size_and_shape__()
        return self

    def diff(self, lag=1, dim=0):
        offs = [[0, 0] for _ in range(self.grid.N_dims)]
        offs[dim] = [0, lag]
        self.diff_op(offs, np.array([-1., 1.]) / (lag * self.grid.delta[dim]))
        self.__update_size_and_shape__()
        return self

    def dzdt(self, lag=1, DOF='dz'):
        self.diff_op(([0, 0], [0, 0], [0, lag]), np.array([-1., 1.]) / (lag * self.grid.delta[2]))
        self.__update_size_and_shape__()
        self.update_dst_grid([0, 0, 0.5 * lag * self.grid.delta[2]], np.array([1, 1, 1]))
        return self

    def d2z_dt2(self, DOF='dz', t_lag=1):
        # the reference returns a NEW operator named 'd2'+DOF+'_dt2' (lin_op.py:286-290)
        op = lin_op(self.grid, name='d2' + DOF + '_dt2').diff_op(
            ([0, 0, 0], [0, 0, 0], [-t_lag, 0, t_lag]), np.array([-1, 2, -1]) / ((t_lag * self.grid.delta[2]) ** 2))
        op.__update_size_and_shape__()
        return op

    # ---- interpolation -----------------------------------------------------------------------
    def interp_mtx(self, pts_in, xform=None, dims=None, bounds_error=True):
        g = self.grid
        if xform is None and g.xform is not None:
            xform = g.xform
        if dims is None:
            dims = np.arange(g.N_dims, dtype=int)
        pts = self.apply_xform(pts_in, xform, dims) if xform is not None else [np.ravel(p) for p in pts_in]
        rows = np.flatnonzero(g.validate_pts(pts))
        if bounds_error and rows.size < len(pts[0]):
            raise ValueError(f'Found {len(pts[0]) - rows.size} points out of bounds for grid {g.name}')
        if rows.size < len(pts[0]):
            pts = [p[rows] for p in pts]
        corners = np.c_[[k.ravel() for k in np.mgrid[tuple(slice(0, 2) for _ in range(g.N_dims))]]] \
            if g.N_dims > 1 else np.array([[0, 1]])
        n_nb, npts = corners.shape[1], rows.size

        def build():   # the triplets on first use (the device path reads only the points)
            fsub = g.float_sub(pts)
            cell = g.cell_sub_for_pts(pts)
            frac = [a - b for a, b in zip(fsub, cell)]
            base = g.global_ind(cell)
            R = np.zeros([npts, n_nb], dtype=int)
            C = np.zeros([npts, n_nb], dtype=int)
            V = np.ones([npts, n_nb], dtype=float)
            for k in range(n_nb):
                R[:, k] = rows
                C[:, k] = base + np.sum(g.stride * corners[:, k])
                for d in range(g.N_dims):
                    V[:, k] *= frac[d] if corners[d, k] else (1. - frac[d])
            return R, C, V, np.arange(0, npts, dtype='int')
        self._lazy = build
        self.N_eq = npts
        self.TOC['rows'] = {self.name: np.arange(self.N_eq, dtype='int')}
        self.TOC['cols'] = {g.name: _grid_cols(g)}
        self.parts = [dict(kind='interp', grid=g, pts=pts, rows=rows, row0=0, n_eq=npts)] \
            if xform is None and bounds_error else None
        self.__update_size_and_shape__()
        return self

    # ---- composition -------------------------------------------------------------------------
    def add(self, op):
        if isinstance(op, (list, tuple)):
            for each in op:
                self.add(each)
            return self
        mine = self._lazy if self._lazy is not None else (lambda a=(self._r, self._c, self._v, self._ind0): a)

        def build(mine=mine, op=op):
            r, c, v, i0 = mine()
            return np.append(r, op.r), np.append(c, op.c), np.append(v, op.v), np.append(i0, op.ind0)
        self._lazy = build
        for key, cols in op.TOC['cols'].items():
            self.TOC['cols'][key] = cols
        self.col_N = np.maximum(self.col_N, op.col_N)
        if self.parts is not None and op.parts is not None:
            self.parts = self.parts + op.parts       # same rows, summed operators
        else:
            self.parts = None
        self.__update_size_and_shape__()
        return self

    def vstack(self, ops, order=None, name=None, TOC_cols=None):
        if isinstance(ops, lin_op):
            ops = (self, ops)
        order = range(len(ops)) if order is None else order
        if name is not None:
            self.name = name
        if TOC_cols is None:
            TOC_cols = {}
            every = []
            for op in ops:
                for key, cols in op.TOC['cols'].items():
                    TOC_cols[key] = cols
                    every.append(np.asarray(cols))
            if self.name is not None:
                TOC_cols[self.name] = _union_sorted(every)
        if self.col_N is None:
            self.col_N = np.max(np.array([op.col_N for op in ops]))
        self.TOC['cols'] = TOC_cols
        ee, parts, offsets = [], [], []
        offset = 0
        for i in order:
            op = ops[i]
            offsets.append((op, offset))
            if op.expected is not None:
                ee.append(np.ravel(op.expected))
            label = op.name if op.name is not None else 'eq'
            base, k = label, 0
            while label in self.TOC['rows']:
                k += 1
                label = f'{base}_{k}'
            if not isinstance(self.TOC['rows'], TocRows):
                self.TOC['rows'] = TocRows(self.TOC['rows'])
            rr = []   # the op's entries, shifted: (first, last) runs or arrays
            for key in list(op.TOC['rows'].keys()):
                kr = toc_range(op.TOC['rows'], key)
                if kr is not None:
                    self.TOC['rows'].set_range(key, kr[0] + offset, kr[1] + 1 + offset)
                    rr.append((kr[0] + offset, kr[1] + offset))
                else:
                    shifted = np.array(op.TOC['rows'][key], dtype='int') + offset
                    self.TOC['rows'][key] = shifted
                    rr.append(shifted.ravel())
            if label not in self.TOC['rows']:
                if all(isinstance(r, tuple) for r in rr) and all(b[0] == a[1] + 1 for a, b in zip(rr, rr[1:])):
                    self.TOC['rows'].set_range(label, rr[0][0], rr[-1][1] + 1)   # consecutive ranges
                else:
                    self.TOC['rows'][label] = np.concatenate(
                        [np.arange(r[0], r[1] + 1) if isinstance(r, tuple) else r for r in rr])
            if parts is not None and op.parts is not None:
                parts.extend(dict(p, row0=p['row0'] + offset) for p in op.parts)
            else:
                parts = None
            offset += op.N_eq
        self.N_eq = offset

        def build(offsets=offsets, ops=tuple(ops)):
            return (np.concatenate([np.ravel(op.r) + off for op, off in offsets]),
                    np.concatenate([np.ravel(op.c) for op, _ in offsets]),
                    np.concatenate([np.ravel(op.v) for op, _ in offsets]),
                    np.concatenate([op.ind0 for op in ops]))
        self._lazy = build
        if ee:
            self.expected = np.concatenate(ee)
        if self.name is not None and len(self.name) > 0:
            self.TOC['rows'].set_range(self.name, 0, offset)
        self.parts = parts
        self.__update_size_and_shape__()
        return self

    # ---- masks, normalisation ----------------------------------------------------------------
    def mask_for_ind0(self, mask_scale=None, mask=None):
        if mask is None:
            mask = self.grid.mask
        if mask is None:
            return np.ones_like(self.ind0, dtype=float)
        flat = np.ravel(mask)
        if flat.size and np.all(flat == flat[0]):
            # uniform mask: every row samples the same value (no need to touch ind0)
            val = flat[0]
            if mask_scale is None:
                return np.full(self.N_eq, val)
            out = np.zeros(self.N_eq, dtype=float)
            for key, scaled in mask_scale.items():
                if val == key:
                    out[:] = scaled
            return out
        rel = self.ind0 - self.grid.col_0
        if len(self.grid.shape) > len(mask.shape):
            subs = tuple(np.unravel_index(rel, self.grid.shape)[:len(mask.shape)])
        else:
            subs = np.unravel_index(rel, mask.shape)
        sampled = mask[subs]
        if mask_scale is None:
            return sampled
        out = np.zeros_like(sampled, dtype=float)
        for key, val in mask_scale.items():
            out[sampled == key] = val
        return out

    def apply_mask(self, mask=None, row_N=None, time_step_overlap=1):
        """Multiply every entry by the mask at its node (lin_op.py:693-732).

        The reference walks the CSR row by row; the product is entry-wise, so here it is one
        gather of the mask on the CSR entries.  Returns the (row, col)-sorted COO of that CSR,
        explicit zeros included, as the reference does.  ``time_step_overlap`` > 1 belongs to
        3-D masks, which lssurf_amd does not support."""
        if time_step_overlap > 1:
            raise NotImplementedError('apply_mask: time_step_overlap (3-D masks) is outside lssurf_amd')
        if mask is None:
            mask = self.grid.mask
        mask = np.asarray(mask)
        A = self.toCSR(row_N=row_N, col_N=self.col_N).tocoo()
        subs = np.unravel_index(A.col - self.grid.col_0, tuple(self.grid.shape))
        A.data = A.data * mask.ravel()[np.ravel_multi_index(list(subs[0:mask.ndim]), mask.shape)]
        self.r, self.c, self.v = A.row, A.col, A.data
        return self

    def apply_2d_mask(self, mask=None):
        """apply_mask with a mask on the first two grid dimensions (lin_op.py:669-691)."""
        if mask is None:
            mask = self.grid.mask
        mask = np.asarray(mask)
        A = self.toCSR().tocoo()
        subs = np.unravel_index(A.col - self.grid.col_0, tuple(self.grid.shape))
        A.data = A.data * mask.ravel()[np.ravel_multi_index([subs[0], subs[1]], mask.shape)]
        self.r, self.c, self.v = A.row, A.col, A.data
        return self

    def mean_of_mask(self, mask, dzdt_lag=None):
        """Area-weighted mean over a 2-D mask (per epoch, or its dz/dt at ``dzdt_lag``),
        lin_op.py:347-402.  ``mask`` is a grid container with ``interp(x, y)``."""
        g = self.grid
        yy, xx = np.meshgrid(g.ctrs[0], g.ctrs[1], indexing='ij')
        mask_g = np.asarray(mask.interp(xx, yy), dtype=float)
        mask_g[~np.isfinite(mask_g)] = 0
        i0, j0 = np.nonzero(mask_g)
        nz = np.flatnonzero(mask_g)
        w = mask_g if g.cell_area is None else mask_g * g.cell_area
        v0 = w.ravel()[nz]
        v0 /= v0.sum()
        y0 = np.sum((g.bds[0][0] + i0.ravel() * g.delta[0]) * v0)
        x0 = np.sum((g.bds[1][0] + j0.ravel() * g.delta[1]) * v0)
        if len(g.shape) < 3:
            # the reference's 2-D branch fails on a misspelt attribute (lin_op.py:374); the
            # single-row operator it means to build is built here
            self.r, self.c, self.v = np.zeros_like(i0), g.global_ind([i0, j0]), v0
            self.N_eq = 1
            self.col_N = np.max(self.c) + 1
            self.__update_size_and_shape__()
            self.dst_grid = fd_grid([[y0, y0], [x0, x0]], g.delta, 0, col_N=0, srs_proj4=g.srs_proj4)
            self.dst_ind0 = np.array([0]).astype(int)
            return self
        nt = int(g.shape[2])
        rr, cc, vv = [], [], []
        if dzdt_lag is None:
            for k in range(nt):
                rr.append(np.zeros_like(i0) + k)
                cc.append(g.global_ind([i0, j0, np.zeros_like(i0) + k]))
                vv.append(v0)
            t_vals = g.ctrs[2]
        else:
            for k in range(nt - dzdt_lag):
                for d_lag in (0, dzdt_lag):
                    rr.append(np.zeros_like(i0) + k)
                    cc.append(g.global_ind([i0, j0, np.zeros_like(i0) + k + d_lag]))
                    vv.append(-v0 / dzdt_lag / g.delta[2] if d_lag == 0 else v0 / d_lag / g.delta[2])
            t_vals = g.ctrs[-1][:-dzdt_lag] + g.delta[-1] * dzdt_lag / 2
        self.r, self.c, self.v = [np.concatenate(a) for a in (rr, cc, vv)]
        self.dst_grid = fd_grid([[y0, y0], [x0, x0], [t_vals[0], t_vals[-1]]], g.delta, 0,
                                col_N=self.r.max() + 1, srs_proj4=g.srs_proj4)
        self.N_eq = self.r.max() + 1
        self.__update_size_and_shape__()
        self.dst_ind0 = np.arange(self.N_eq, dtype=int)
        return self

    def normalize_by_unit_product(self, wt=1):
        absop = lin_op(col_N=self.col_N)
        absop.N_eq = self.N_eq
        absop.r, absop.c, absop.v = self.r, self.c, np.abs(self.v)
        absop.__update_size_and_shape__()
        norm = absop.toCSR(row_N=absop.N_eq).dot(np.ones(self.shape[1]))
        scale = np.zeros_like(norm)
        scale[norm > 0] = 1. / norm[norm > 0]
        self.v *= scale[self.r] * wt
        self.parts = None

    def sum_to_grid3(self, kernel_size, sub0s=None, lag=None, taper=True, valid_equations_only=True, dims=None):
        """Sum (tapered) blocks of nodes onto a coarser output grid (lin_op.py:404-488)."""
        g = self.grid
        kernel_size = np.asarray(kernel_size)
        half = np.floor((kernel_size - 1) / 2).astype(int) if taper else np.floor(kernel_size / 2).astype(int)
        dims = list(range(len(g.shape))) if dims is None else list(dims)
        nd = len(dims)
        if sub0s is None:
            if taper and valid_equations_only:
                axes = [np.arange(half[i] + 1, g.shape[i], kernel_size[i] - 1, dtype=int) for i in dims]
            elif taper:
                axes = [np.arange(0, g.shape[i] + 1, kernel_size[i] - 1, dtype=int) for i in dims]
            else:
                axes = [np.arange(half[i], g.shape[i], kernel_size[i], dtype=int) for i in dims]
            sub0s = np.meshgrid(*axes, indexing='ij')
        ind0 = g.global_ind(sub0s[0:nd])
        if np.mod(kernel_size[0] / 2, 1) == 0:
            di, dj = np.meshgrid(np.arange(-half[0], half[0]), np.arange(-half[1], half[1]), indexing='ij')
            grid_shift = [-g.delta[0] / 2, -g.delta[1] / 2, 0][0:nd]
        else:
            di, dj = np.meshgrid(np.arange(-half[0], half[0] + 1), np.arange(-half[1], half[1] + 1), indexing='ij')
            grid_shift = [0, 0, 0][0:nd]
        w0 = np.ones(kernel_size[0:2], dtype=float)
        if taper:
            for edge in (0, -1):
                w0[edge, :] /= 2
                w0[:, edge] /= 2
        w0 = w0.ravel()
        di, dj = di.ravel(), dj.ravel()
        if lag is None:
            offsets = [di, dj, np.zeros_like(di)]
            wt = w0
            grid_shift = [0, 0, 0]
        else:
            offsets = [np.concatenate([di, di]), np.concatenate([dj, dj]),
                       np.concatenate([np.zeros_like(di, dtype=int), np.zeros_like(di, dtype=int) + lag])]
            wt = np.concatenate([-w0, w0]) / (lag * g.delta[2])
            grid_shift[2] = 0.5 * lag * g.delta[2]
        self.diff_op(offsets, wt.astype(float), which_nodes=ind0, valid_equations_only=valid_equations_only)
        self.update_dst_grid(grid_shift, np.maximum(1, kernel_size - 1) if taper else kernel_size)
        return self

    def update_dst_grid(self, grid_shift, kernel_size):
        rcv0 = np.unravel_index(self.ind0 - self.grid.col_0, self.grid.shape)
        dims = range(len(self.grid.shape))
        bounds = [[self.grid.ctrs[d][rcv0[d][j]] + grid_shift[d] for j in (0, -1)] for d in dims]
        self.dst_grid = fd_grid(bounds, kernel_size * self.grid.delta, name=self.name)
        out_subs = [((rcv0[d] - rcv0[d][0]) / kernel_size[d]).astype(int) for d in dims]
        self.dst_ind0 = np.ravel_multi_index(out_subs, self.dst_grid.shape)
        return self

    def data_bias(self, ind=None, val=None, col=None, DOF=None):
        if col is None:
            col = self.col_N
            self.col_N += 1
        self.r = ind
        self.c = np.zeros_like(ind, dtype='int') + col
        self.v = np.ones_like(ind, dtype='float') if val is None else val.ravel()
        self.TOC['rows'] = {self.name: np.unique(self.r)}
        self.TOC['cols'] = {self.name: np.unique(self.c)}
        self.N_eq = np.max(ind) + 1
        self.parts = None
        self.__update_size_and_shape__()
        return self

    # ---- products on solutions ---------------------------------------------------------------
    def _out_grid_and_rows(self, grid):
        if grid is None:
            grid = self.grid if self.dst_grid is None else self.dst_grid
        rows = self.ind0 if self.dst_ind0 is None else self.dst_ind0
        return grid, rows

    def grid_prod(self, m, grid=None):
        grid, rows = self._out_grid_and_rows(grid)
        P = np.zeros(grid.col_N + 1) + np.nan
        P[rows] = self.toCSR(row_N=rows.size, col_N=m.size).dot(m).ravel()
        return P[grid.col_0:grid.col_N].reshape(grid.shape)

    def grid_error(self, Rinv, grid=None):
        grid, rows = self._out_grid_and_rows(grid)
        E = np.zeros(self.col_N) + np.nan
        E[rows] = np.sqrt((self.toCSR(row_N=rows.size, col_N=Rinv.shape[0]).dot(Rinv)).power(2).sum(axis=1)).ravel()
        return E[grid.col_0:grid.col_N].reshape(grid.shape)

    def print_TOC(self):
        for rc in ('cols', 'rows'):
            print(rc)
            first = {k: np.min(self.TOC[rc][k]) for k in self.TOC[rc]}
            for key in sorted(first, key=first.get):
                print('\t%s\t%d : %d' % (key, np.min(self.TOC[rc][key]), np.max(self.TOC[rc][key])))

    def toCSR(self, col_N=None, row_N=None):
        if col_N is None:
            col_N = self.col_N
        self.fix_dtypes()
        nz = np.ravel(self.v) != 0
        r = np.ravel(self.r)[nz]
        if row_N is None:
            row_N = np.max(r) + 1
        return sp.csr_matrix((np.ravel(self.v)[nz], (r, np.ravel(self.c)[nz])), shape=(row_N, col_N))

    def triplets(self):
        """(r, c, v) flattened, int64/int64/float64 — the COO handed to the device."""
        return (np.ravel(self.r).astype(np.int64), np.ravel(self.c).astype(np.int64),
                np.ravel(self.v).astype(np.float64))
