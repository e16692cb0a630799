"""Regular N-D finite-difference grid: node layout and global column indexing.

Restates LSsurf/fd_grid.py:13-145 (class ``fd_grid``): node count per dimension
``int((b1-b0)/delta + 1)`` (fd_grid.py:61), node centres ``b0 + delta*arange(N)`` (:62),
row-major strides (:67) and global column index ``col_0 + ravel_multi_index(sub, shape)``
(:130-145).  Points are validated inclusively against the first/last node (:90-96); the cell of
a point is ``floor((p - b0)/delta)`` (:120-128).  The device assembler (lssurf_amd/csrc) uses
exactly these formulas.  Mask *files* (GeoTIFF / vector via GDAL, fd_grid.py:147-198) are out
of scope; in-memory masks (ndarray or grid objects with ``interp``) are supported.
"""
import copy as _copy

import numpy as np


class fd_grid:
    def __init__(self, bounds, deltas, name='', col_0=0, col_N=None, srs_proj4=None, mask_file=None,
                 mask_data=None, mask_interp_threshold=0.5, erode_source_mask=True, xform=None,
                 coords=('y', 'x', 'time')):
        self.delta = np.array(deltas)
        n_per_dim = [((hi_lo[1] - hi_lo[0]) / d) + 1 for hi_lo, d in zip(bounds, self.delta)]
        self.shape = np.array(n_per_dim).astype(int)
        self.ctrs = [lo_hi[0] + d * np.arange(n) for lo_hi, d, n in zip(bounds, self.delta, self.shape)]
        self.bds = [np.array([c[0], c[-1]]) for c in self.ctrs]
        self.N_dims = len(self.shape)
        self.N_nodes = np.prod(self.shape)
        # stride[k] = number of nodes spanned by one step in dimension k (row-major)
        self.stride = np.array([np.prod(self.shape[k + 1:]) for k in range(self.N_dims)], dtype=int)
        self.col_0 = col_0
        self.col_N = self.col_0 + self.N_nodes if col_N is None else col_N
        self.srs_proj4 = srs_proj4
        self.name = name
        self.coords = list(coords)
        self.user_data = {}
        self.xform = xform
        self.cell_area = None
        self.mask_interp_threshold = mask_interp_threshold
        self.erode_source_mask = erode_source_mask
        self.mask = np.ones(self.shape[0:2], dtype=bool)
        self.mask_3d = None
        self.mask_file = None
        if mask_file is not None and mask_data is None:
            raise NotImplementedError('fd_grid: mask files (GDAL I/O) are outside lssurf_amd; pass mask_data')
        if mask_data is not None:
            self.setup_mask(mask_data=mask_data, interp_threshold=mask_interp_threshold)

    def copy(self):
        return _copy.deepcopy(self)

    # ---- masks (in-memory only) --------------------------------------------------------------
    def setup_mask(self, mask_data=None, mask_file=None, interp_threshold=0.5):
        if mask_file is not None:
            raise NotImplementedError('fd_grid: mask files are outside lssurf_amd')
        if mask_data is None:
            return
        if isinstance(mask_data, np.ndarray):
            self.mask = mask_data.astype(bool)
            if mask_data.ndim > 2:
                self.mask_3d = mask_data.astype(bool)
            return
        if len(getattr(mask_data, 'shape', ())) > 2:
            raise NotImplementedError('fd_grid: time-varying grid masks are outside lssurf_amd')
        self.mask = mask_data.interp(self.ctrs[1], self.ctrs[0], gridded=True) > interp_threshold

    # ---- point / node geometry ---------------------------------------------------------------
    def validate_pts(self, pts):
        inside = np.isfinite(pts[0])
        for dim in range(self.N_dims):
            lo, hi = self.bds[dim]
            with np.errstate(invalid='ignore'):
                inside &= (pts[dim] >= lo) & (pts[dim] <= hi)
        return inside

    def float_sub(self, pts, good=None):
        if good is None:
            good = self.validate_pts(pts)
        out = []
        for dim in range(len(pts)):
            sub = np.full(np.shape(pts[0]), np.nan)
            if dim < self.N_dims:
                sub[good] = (pts[dim][good] - self.bds[dim][0]) / self.delta[dim]
            out.append(sub)
        return out

    def cell_sub_for_pts(self, pts, good=None):
        if good is None:
            good = self.validate_pts(pts)
        out = []
        for dim in range(len(pts)):
            sub = np.full(np.shape(pts[0]), np.nan)
            if dim < self.N_dims:
                sub[good] = np.floor((pts[dim][good] - self.bds[dim][0]) / self.delta[dim])
            out.append(sub)
        return out

    def global_ind(self, cell_sub, return_valid=False):
        subs = [np.asarray(s).astype(int) for s in cell_sub]
        if not return_valid:
            return self.col_0 + np.ravel_multi_index(subs, self.shape)
        ok = np.ones_like(subs[0], dtype=bool)
        for dim, s in enumerate(subs):
            ok &= (s >= 0) & (s < self.shape[dim])
        ind = np.zeros_like(subs[0])
        ind[ok] = self.col_0 + np.ravel_multi_index([s[ok] for s in subs], self.shape)
        return ind, ok

    def pos_for_nodes(self, nodes):
        subs = np.unravel_index(nodes, self.shape)
        return [s * d + b[0] for d, b, s in zip(self.delta, self.bds, subs)]

    def get_extent(self, dims=(1, 0)):
        return np.concatenate([self.bds[d] + self.delta[d] * np.array([-0.5, 0.5]) for d in dims])

    def __repr__(self):
        return f'fd_grid(name={self.name!r}, shape={tuple(self.shape)}, col_0={self.col_0}, col_N={self.col_N})'
