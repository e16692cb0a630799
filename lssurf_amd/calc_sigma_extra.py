"""Robust spread and the extra data error used by smooth_fit's outlier editing.

Mirror of LSsurf/RDE.py:10-18 and LSsurf/calc_sigma_extra.py:13-109.  With `device` set, the
25–30 RDE evaluations of calc_sigma_extra's bounded search sort on the GPU (liblsqsurf
lsq_rde_*): r and σ are uploaded once per group, each evaluation
returns only the four order statistics numpy's interpolation needs, and the interpolation and
scipy's bounded Brent search run unchanged on the host — the result is bit-identical to the
host path (tests/test_gpu_smooth_fit.py).
"""
import ctypes

import numpy as np
import scipy.optimize as scipyo


def RDE(x):
    """Half the 16–84 percentile spread of the finite values (linear interpolation on
    mid-rank positions 0.5, 1.5, ...), NaN with fewer than two finite values."""
    finite = np.isfinite(x)
    n = int(np.sum(finite))
    if n < 2:
        return np.nan
    lo, hi = np.interp(np.array([0.16, 0.84]) * n, np.arange(0.5, n), np.sort(x[finite]))
    return (hi - lo) / 2.


class DeviceRDE:
    """RDE(r / sqrt(s² + σ²)) on the device for a fixed (r, σ); bit-identical to
    RDE(r / np.sqrt(s ** 2 + sigma ** 2)) on the host."""

    def __init__(self, r, sigma, device=0):
        from ._native import NativeError, load, ptr
        self._L, self._ptr = load(), ptr
        r = np.ascontiguousarray(r, dtype=np.float64)
        sigma = np.ascontiguousarray(sigma, dtype=np.float64)
        keep = np.isfinite(r) & np.isfinite(sigma)
        self.r, self.sigma = r[keep], sigma[keep]
        self.n = int(self.r.size)
        self._c = None
        if self.n >= 2:
            self._c = self._L.lsq_rde_create(int(device), self.n, ptr(self.r), ptr(self.sigma))
            if not self._c:
                raise NativeError('lsq_rde_create failed (no gfx950 device?)')

    def __call__(self, s):
        n = self.n
        if n < 2 or not np.isfinite(s):
            return RDE(self.r / np.sqrt(s ** 2 + self.sigma ** 2))   # degenerate: host path
        q = np.array([0.16, 0.84]) * n
        j = np.clip(np.floor(q - 0.5).astype(np.int64), 0, n - 2)
        idx = np.ascontiguousarray(np.stack([j, j + 1], axis=1).ravel(), dtype=np.int64)
        v = np.zeros(4)
        if self._L.lsq_rde_order_stats(self._c, float(s), 4, self._ptr(idx), self._ptr(v)) != 0:
            from ._native import NativeError
            raise NativeError(self._L.lsq_rde_last_error(self._c).decode())
        # np.interp on the two bracketing mid-rank positions = np.interp on all of them
        lo = np.interp(q[0], j[0] + np.array([0.5, 1.5]), v[0:2])
        hi = np.interp(q[1], j[1] + np.array([0.5, 1.5]), v[2:4])
        return (hi - lo) / 2.

    def close(self):
        if self._c:
            self._L.lsq_rde_destroy(self._c)
            self._c = None

    def __del__(self):
        self.close()


def calc_sigma_extra(r, sigma, mask, sigma_extra_masks=None, device=None):
    """sigma_extra such that RDE(r / sqrt(sigma² + sigma_extra²)) == 1 (bounded scalar search
    on [0, RDE(r)]), per sigma_extra mask; groups with < 10 selected points get 0.  With
    `device` (GPU ordinal) the RDE evaluations sort on the device (same result)."""
    if sigma_extra_masks is None:
        sigma_extra_masks = {'all': np.ones_like(r, dtype=bool)}
    out = np.zeros_like(r)
    for group in sigma_extra_masks.values():
        sel = group & mask
        if np.sum(sel) < 10:
            continue
        rr, ss = r[sel], sigma[sel]
        if device is not None and np.all(np.isfinite(rr)) and np.all(np.isfinite(ss)):
            drde = DeviceRDE(rr, ss, device)
            cost = lambda s1: (drde(s1) - 1) ** 2  # noqa: E731
        else:
            drde = None
            cost = lambda s1: (RDE(rr / np.sqrt(s1 ** 2 + ss ** 2)) - 1) ** 2  # noqa: E731
        try:
            out[group] = scipyo.minimize_scalar(cost, method='bounded', bounds=[0, RDE(rr)])['x']
        except Exception as err:   # the reference prints and continues (calc_sigma_extra.py:42-43)
            print(err)
        finally:
            if drde is not None:
                drde.close()
    return out


def calc_sigma_extra_on_grid(x, y, r, sigma, in_TSE, sigma_extra_masks=None, spacing=1.e4, L_avg=None,
                             sigma_extra_max=None):
    """Tent-weighted blend of sigma_extra estimated in overlapping square bins."""
    L_avg = 2 * spacing if L_avg is None else L_avg
    full = calc_sigma_extra(r, sigma, in_TSE, sigma_extra_masks=sigma_extra_masks)
    centres = np.unique(np.round((x + 1j * y) / spacing) * spacing)
    wsum = np.zeros_like(r)
    wsig = np.zeros_like(r)
    half = L_avg / 2
    for c in centres:
        dx, dy = np.abs(np.real(c) - x), np.abs(np.imag(c) - y)
        inside = (dx < half) & (dy < half)
        sel = in_TSE & inside
        if np.sum(sel) < 10:
            continue
        s = calc_sigma_extra(r, sigma, sel, sigma_extra_masks=sigma_extra_masks)
        if sigma_extra_max is not None:
            s = np.minimum(s, sigma_extra_max)
        W = inside * (1 - dx / half) * (1 - dy / half)
        wsig += W * s
        wsum += W
    out = np.zeros_like(r) + full
    has = wsum > 0
    out[has] = wsig[has] / wsum[has]
    return out
