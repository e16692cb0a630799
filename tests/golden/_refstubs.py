"""Minimal stand-ins that let the *reference* LSsurf package import in the survey container.

Used only by tests/golden/gen_golden.py (fixture generation; never shipped, never run on the
GPU box).  The reference imports pointCollection, osgeo, geopandas and PySPQR at module level
(LSsurf/smooth_fit.py:16-19, fd_grid.py:9, setup_DEM_jitter_fit.py:14); none is installed.

* pointCollection.data / grid.data: duck-typed point and grid containers with exactly the
  members the solve path touches (from_dict, from_list, coords, copy_subset, index, assign,
  copy, fields, size, shape, __getitem__).
* sparseqr.solve / sparseqr.rz: the exact dense least-squares oracle (oracle/dense.py); every
  call records its (A, b) so the generator can store the exact matrix the reference formed.
* LSsurf.inv_tr_upper etc.: the reference's own Cython kernels compiled by oracle/build_ref.sh.
"""
import importlib.util
import os
import sys
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = '/root/reference'
CALLS = []          # (A_coo, b) recorded for every sparseqr.solve call
RZ_CALLS = []       # A recorded for every sparseqr.rz call (compute_E)
SOLS = []           # the exact solution returned by every sparseqr.solve call


def sp_csr(A):
    import scipy.sparse as sp
    return sp.csr_matrix(A).copy()


class _PcData:
    def __init__(self):
        self.fields = []
        self.size = 0
        self.shape = (0,)

    def _upd(self):
        if self.fields:
            a = getattr(self, self.fields[0])
            self.size, self.shape = a.size, a.shape

    def from_dict(self, d):
        for k, v in d.items():
            setattr(self, k, np.asarray(v))
            if k not in self.fields:
                self.fields.append(k)
        self._upd()
        return self

    def from_list(self, lst):
        fields = lst[0].fields
        return _PcData().from_dict({f: np.concatenate([getattr(D, f).ravel() for D in lst])
                                    for f in fields})

    def copy(self):
        return _PcData().from_dict({f: getattr(self, f).copy() for f in self.fields})

    def copy_subset(self, idx):
        return _PcData().from_dict({f: getattr(self, f)[idx] for f in self.fields})

    def __getitem__(self, idx):
        return self.copy_subset(idx)

    def index(self, idx):
        for f in self.fields:
            setattr(self, f, getattr(self, f)[idx])
        self._upd()
        return self

    def assign(self, d=None, **kw):
        if d is None:
            d = {}
        d = dict(d, **kw)
        return self.from_dict(d)

    def coords(self):
        c = [self.y, self.x]
        if 'time' in self.fields:
            c.append(self.time)
        return c


class _PcGrid(_PcData):
    def interp(self, x, y, gridded=False, field='z'):
        """bilinear interpolation on the node lattice (x, y vectors); NaN outside.  The
        averaging-mask fixtures sample it at its own nodes, where any bilinear scheme is exact."""
        z = np.asarray(getattr(self, field), float)
        gx, gy = np.asarray(self.x, float), np.asarray(self.y, float)
        x, y = np.asarray(x, float), np.asarray(y, float)
        fx, fy = np.interp(x, gx, np.arange(gx.size)), np.interp(y, gy, np.arange(gy.size))
        i = np.clip(np.floor(fy).astype(int), 0, gy.size - 2)
        j = np.clip(np.floor(fx).astype(int), 0, gx.size - 2)
        a, b = fy - i, fx - j
        out = (z[i, j] * (1 - a) * (1 - b) + z[i + 1, j] * a * (1 - b) + z[i, j + 1] * (1 - a) * b
               + z[i + 1, j + 1] * a * b)
        out[(x < gx[0]) | (x > gx[-1]) | (y < gy[0]) | (y > gy[-1])] = np.nan
        return out


class _PcGridRBS(_PcGrid):
    def interp(self, x, y, gridded=False, field='z'):
        """pointCollection.grid.data.interp for the anisotropic notebook's direction field: a
        bilinear RectBivariateSpline (kx = ky = 1) evaluated at the points (y, x)."""
        from scipy.interpolate import RectBivariateSpline
        z = np.asarray(getattr(self, field), float)
        f = RectBivariateSpline(np.asarray(self.y, float), np.asarray(self.x, float), z, kx=1, ky=1)
        return f.ev(np.asarray(y, float), np.asarray(x, float))


def install():
    """Install the stubs and register the compiled reference kernels; returns LSsurf."""
    if not os.path.isdir(REF):
        raise RuntimeError('reference absent')
    for name in ['osgeo', 'osgeo.osr', 'osgeo.ogr', 'geopandas', 'requests',
                 'pointCollection', 'pointCollection.grid', 'sparseqr', 'PointDatabase']:
        sys.modules.setdefault(name, types.ModuleType(name))
    g = types.ModuleType('osgeo.gdal')
    g.GDT_Float32, g.GRA_NearestNeighbour, g.GRA_Average = 6, 0, 5
    sys.modules['osgeo.gdal'] = g
    osgeo = sys.modules['osgeo']
    osgeo.gdal, osgeo.osr, osgeo.ogr = g, sys.modules['osgeo.osr'], sys.modules['osgeo.ogr']
    pc = sys.modules['pointCollection']
    pc.data = _PcData
    pc.grid = sys.modules['pointCollection.grid']
    pc.grid.data = _PcGrid

    sys.path.insert(0, REPO)
    from oracle import dense
    sq = sys.modules['sparseqr']

    def solve(A, b, tolerance=None):
        CALLS.append((A.tocsr().copy(), np.array(b, dtype=float).copy()))
        x = dense.ls_solve_dense(A, b)
        SOLS.append(x.copy())
        return x
    sq.solve = solve

    def rz(A, b):
        RZ_CALLS.append(sp_csr(A))
        return dense.rz_dense(A, b)
    sq.rz = rz

    # reference Cython kernels (built from /root/reference/LSsurf/*.pyx by oracle/build_ref.sh)
    np.float = float   # propagate_qz_errors.pyx:7 / spsolve_tr_upper.pyx:6 use the removed alias
    refdir = os.path.join(REPO, 'oracle', '_ref')
    for k in ['inv_tr_upper', 'propagate_qz_errors', 'spsolve_tr_upper']:
        so = [f for f in os.listdir(refdir) if f.startswith(k + '.') and f.endswith('.so')][0]
        spec = importlib.util.spec_from_file_location(k, os.path.join(refdir, so))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules['LSsurf.' + k] = mod
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import LSsurf
    return LSsurf
