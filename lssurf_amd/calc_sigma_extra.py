"""Robust spread and the extra data error used by smooth_fit's outlier editing.

Host mirror of LSsurf/RDE.py:10-18 and LSsurf/calc_sigma_extra.py:13-109 (numpy/scipy; moving
this to the device is §8(f) "next" row 1).
"""
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


def calc_sigma_extra(r, sigma, mask, sigma_extra_masks=None):
    """sigma_extra such that RDE(r / sqrt(sigma² + sigma_extra²)) == 1 (bounded scalar search
    on [0, RDE(r)]), per sigma_extra mask; groups with < 10 selected points get 0."""
    if sigma_extra_masks is None:
        sigma_extra_masks = {'all': np.ones_like(r, dtype=bool)}
    out = np.zeros_like(r)
    for group in sigma_extra_masks.values():
        sel = group & mask
        if np.sum(sel) < 10:
            continue
        rr, ss = r[sel], sigma[sel]
        cost = lambda s1: (RDE(rr / np.sqrt(s1 ** 2 + ss ** 2)) - 1) ** 2  # noqa: E731
        try:
            out[group] = scipyo.minimize_scalar(cost, method='bounded', bounds=[0, RDE(rr)])['x']
        except Exception as err:   # the reference prints and continues (calc_sigma_extra.py:42-43)
            print(err)
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
