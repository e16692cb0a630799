"""Duck-typed point and grid containers with the interface the solve path uses from the
external ``pointCollection`` package (pc.data at LSsurf/smooth_fit.py:406-433,658-662;
pc.grid.data at smooth_fit.py:257-263,279-298).  Any object with the same members works as
input to ``smooth_fit``; these are what the outputs are built from.

Usage mirrors pointCollection::

    from lssurf_amd import containers as pc
    D = pc.data().from_dict({'x': x, 'y': y, 'time': t, 'z': z, 'sigma': s})
    G = pc.grid.data().from_dict({'x': xc, 'y': yc, 'z0': z0})
"""
import types

import numpy as np


class PointData:
    """Columns of equal-length arrays; ``coords()`` returns (y, x[, time])."""

    def __init__(self, fields=None):
        self.fields = []
        self.size = 0
        self.shape = (0,)
        if fields:
            self.from_dict(fields)

    def _sync(self):
        if self.fields:
            first = getattr(self, self.fields[0])
            self.size, self.shape = first.size, first.shape
        return self

    def from_dict(self, d):
        for key, val in d.items():
            setattr(self, key, np.asarray(val))
            if key not in self.fields:
                self.fields.append(key)
        return self._sync()

    def from_list(self, items):
        keys = items[0].fields
        return type(self)().from_dict({k: np.concatenate([np.ravel(getattr(it, k)) for it in items]) for k in keys})

    def assign(self, d=None, **kw):
        merged = dict(d or {})
        merged.update(kw)
        return self.from_dict(merged)

    def copy(self):
        return type(self)().from_dict({k: np.copy(getattr(self, k)) for k in self.fields})

    def copy_subset(self, index):
        return type(self)().from_dict({k: getattr(self, k)[index] for k in self.fields})

    def __getitem__(self, index):
        return self.copy_subset(index)

    def index(self, index):
        for k in self.fields:
            setattr(self, k, getattr(self, k)[index])
        return self._sync()

    def coords(self):
        out = [self.y, self.x]
        for tname in ('time', 't'):
            if tname in self.fields:
                out.append(getattr(self, tname))
                break
        return out

    def __repr__(self):
        return f'{type(self).__name__}(size={self.size}, fields={self.fields})'


class GridData(PointData):
    """Gridded fields with 1-D coordinate vectors x, y (and optionally time / t)."""

    def _sync(self):
        for k in self.fields:
            if k not in ('x', 'y', 't', 'time'):
                a = getattr(self, k)
                if a is not None and np.ndim(a) >= 2:
                    self.shape, self.size = a.shape, a.size
                    break
        return self

    def interp(self, x, y, gridded=False, field='z'):
        """Bilinear interpolation of ``field`` at (x, y); NaN outside the grid."""
        z = getattr(self, field)
        if gridded:
            xx, yy = np.meshgrid(x, y)
        else:
            xx, yy = np.asarray(x, float), np.asarray(y, float)
        gx, gy = np.asarray(self.x, float), np.asarray(self.y, float)
        fx = (xx - gx[0]) / (gx[1] - gx[0]) if gx.size > 1 else np.zeros_like(xx)
        fy = (yy - gy[0]) / (gy[1] - gy[0]) if gy.size > 1 else np.zeros_like(yy)
        ix = np.clip(np.floor(fx).astype(int), 0, max(gx.size - 2, 0))
        iy = np.clip(np.floor(fy).astype(int), 0, max(gy.size - 2, 0))
        wx, wy = fx - ix, fy - iy
        ix1, iy1 = np.minimum(ix + 1, gx.size - 1), np.minimum(iy + 1, gy.size - 1)
        zf = np.asarray(z, float)
        out = (zf[iy, ix] * (1 - wx) * (1 - wy) + zf[iy, ix1] * wx * (1 - wy) + zf[iy1, ix] * (1 - wx) * wy
               + zf[iy1, ix1] * wx * wy)
        bad = (fx < 0) | (fx > gx.size - 1) | (fy < 0) | (fy > gy.size - 1)
        out = np.where(bad, np.nan, out)
        return out


data = PointData
grid = types.SimpleNamespace(data=GridData)
