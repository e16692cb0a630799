"""The anisotropic-constraint systems of notebooks/smooth_fit_demo_aniso.ipynb (BASELINE config C5).

* ``directional_smoothing_op`` — notebook cell 10 (with cells 8-9): the second derivative
  along a direction field u, d2z/dx2·u² + 2·d2z/dxdy·u·v + d2z/dy2·v², built from three
  lin_op.diff_op templates padded to the union of their offsets (cell 8) whose rows are scaled
  by the field interpolated at each row's centre (cell 9).  The row scaling keeps the lin_op
  structure (lin_op.scale_rows / scale_values), so the operator is formed on the device as one
  field-valued stencil part (lsq_set_stencil_fields) — triplets identical to the reference's.
* ``system`` — the 2-D notebook system handed to ``sparseqr.solve`` (cells 13-18): z0 grid on
  [-10, 10]², data rows, Axy (E = 0.25) and the magnitude constraint (expected 2), as COO.
* ``system3d`` — config C5: the smooth_fit z0 + dz system (SURVEY.md §8(d) synthetic setup) with
  the z0 smoothness constraints replaced by Axy and the magnitude constraint.

The direction field is interpolated as pointCollection.grid.data.interp does (bilinear
RectBivariateSpline, kx = ky = 1; pointCollection is an unversioned git dependency absent here,
so this restatement is what tests/golden/gen_golden.py uses for the reference run too).
"""
import numpy as np
import scipy.sparse as sp
from scipy.interpolate import RectBivariateSpline

from . import containers as pc
from .fd_grid import fd_grid
from .lin_op import lin_op


def interp_field(u, x, y, field):
    """pointCollection.grid.data.interp(x, y, field=field) for a 2-D field on ascending x, y."""
    z = np.asarray(getattr(u, field), dtype=float)
    return RectBivariateSpline(np.asarray(u.y, float), np.asarray(u.x, float), z, kx=1, ky=1).ev(
        np.asarray(y, float), np.asarray(x, float))


def _row_centres(op):
    """notebook cell 9: node coordinates of each row's ind0 (diff_op rows: the centre node)."""
    temp = list(np.unravel_index(op.ind0 - op.grid.col_0, op.grid.shape))
    for dim in range(len(temp)):
        temp[dim] = op.grid.bds[dim][0] + op.grid.delta[dim] * temp[dim]
        if temp[dim].ndim > 1:
            temp[dim] = np.mean(temp[dim], axis=1)
    return temp


def _scale_op_by_2d_grid(op, data_grid, field, power=None):
    """notebook cell 9: scale each row by `field` interpolated at the row's node position."""
    temp = _row_centres(op)
    zi = interp_field(data_grid, temp[1], temp[0], field)
    if power is not None:
        zi = zi ** power
    return op.scale_rows(zi)


def _system_of_ops(stencils):
    """notebook cell 8: give every stencil the union of the offsets (zero coefficients added).
    The union is walked in Python set order, as the notebook does."""
    offsets = set()
    for st in stencils.values():
        this = set(tuple(jj) for jj in zip(*st[0]))
        offsets.update(this)
    for st in stencils.values():
        st[1] = list(st[1])
        have = set(tuple(jj) for jj in zip(*st[0]))
        for off in offsets:
            if off not in have:
                for dim, oo in enumerate(off):
                    st[0][dim].append(oo)
                st[1].append(0)
        st[1] = np.array(st[1])


def directional_smoothing_op(grid, u):
    """notebook cell 10."""
    coeffs = np.array([-1., 2., -1.]) / (grid.delta[0] ** 2)
    stencils = {'d2zdx2': [([0, 0, 0], [-1, 0, 1]), coeffs],
                'd2zdy2': [([-1, 0, 1], [0, 0, 0]), coeffs],
                'd2zdxdy': [([-1, -1, 1, 1], [-1, 1, -1, 1]), np.array([-1., 1., 1., -1]) / (4 * grid.delta[0] ** 2)]}
    for st in stencils.values():
        st[0] = tuple(list(d) for d in st[0])
    _system_of_ops(stencils)
    Axy = lin_op(grid=grid).diff_op(*stencils['d2zdx2'])
    _scale_op_by_2d_grid(Axy, u, 'u', power=2)
    temp = lin_op(grid=grid).diff_op(*stencils['d2zdxdy'])
    _scale_op_by_2d_grid(temp, u, 'v')
    _scale_op_by_2d_grid(temp, u, 'u')
    temp.scale_values(2)
    Axy.add(temp)
    temp = lin_op(grid=grid).diff_op(*stencils['d2zdy2'])
    _scale_op_by_2d_grid(temp, u, 'v', power=2)
    Axy.add(temp)
    return Axy


def circular_field(step=0.125, half_width=10.):
    """notebook cell 15: unit vectors around the origin on a [-10, 10]² lattice of `step`,
    coordinates scaled to [-half_width, half_width] (the field is scale-free: np.gradient works
    in index units)."""
    xg, yg = np.meshgrid(np.arange(-10, 10.01, step), np.arange(-10, 10.01, step))
    zg = np.abs(xg + 1j * yg)
    vp, up = np.gradient(zg)
    uv = 1j * (up + 1j * vp)
    uv[np.abs(uv) == 0] = 1
    uv /= np.abs(uv)
    s = half_width / 10.
    return pc.grid.data().from_dict({'x': xg[0, :] * s, 'y': yg[:, 0] * s, 'u': np.real(uv), 'v': np.imag(uv)})


def system_ops(nodes=401, npts=0, seed=20251121 + 5, E_aniso=0.25, mag_expected=2.0, u=None, pts=None):
    """The notebook system as lin_ops: (G_data, Gc, E, rhs, grid) — z0 grid with `nodes` per side
    on [-10, 10]² (the notebook: 401), data rows, Gc = [Axy; mag_z0] (cells 13-18), σ and rhs.
    pts = (x, y, z) overrides the points (default: `npts` synthetic ones, or the notebook's eight
    points on a circle, cell 18)."""
    delta = 20. / (nodes - 1)
    g = fd_grid([[-10., 10.], [-10., 10.]], delta * np.ones(2), name='z0')
    rng = np.random.default_rng(seed)
    if pts is not None:
        x, y, z = (np.asarray(a, float) for a in pts)
    elif npts:
        x, y = rng.uniform(-10, 10, npts), rng.uniform(-10, 10, npts)
        z = 10 * np.sin(2 * np.pi * x / 10) * np.cos(2 * np.pi * y / (20 / 3)) + rng.normal(0, 0.1, npts)
    else:     # the notebook's eight points on a circle (cell 18)
        pp = 5 * np.exp(1j * np.arange(0, 2 * np.pi, np.pi / 4))
        x, y, z = np.real(pp), np.imag(pp), np.ones(pp.size)
    sigma = np.full(x.size, 0.1)
    G_data = lin_op(g, name='interp_z').interp_mtx([y, x])
    Axy = directional_smoothing_op(g, circular_field() if u is None else u)
    Axy.expected = E_aniso + np.zeros(Axy.N_eq)
    mag = lin_op(g, name='mag_z0').one(DOF='z0')
    mag.expected = mag_expected + np.zeros(mag.N_eq)
    Gc = lin_op(None, name='constraints').vstack([Axy, mag])
    E = np.concatenate([sigma, Axy.expected, mag.expected])
    rhs = np.concatenate([z, np.zeros(Gc.N_eq)])
    return G_data, Gc, E, rhs, g


def system(*args, **kw):
    """(A, b, grid) with A = TCinv·[G_data; Axy; mag_z0] (COO) and b = TCinv·rhs, as the notebook
    passes them to sparseqr.solve (system_ops' arguments)."""
    G_data, Gc, E, rhs, g = system_ops(*args, **kw)
    G = sp.vstack([G_data.toCSR(), Gc.toCSR()]).tocsr()
    A = (sp.diags(1. / E) @ G).tocoo()
    return A, (1. / E) * rhs, g      # TCinv.dot(rhs)


def aniso_expected(E_RMS, grid):
    """σ of the directional rows in the 3-D system: the σ smooth_fit gives the isotropic
    grad2_z0 rows it replaces (E_RMS['d2z0_dx2'] / sqrt(cell area), constraint_functions.py:42-44)."""
    return E_RMS['d2z0_dx2'] / np.sqrt(np.prod(grid.delta))


def system3d(data, W, ctr, spacing, E_RMS, reference_epoch=0, u=None, E_aniso=None, mag_expected=2.0, **kw):
    """Config C5: smooth_fit's z0 + dz system with z0's smoothness constraints (grad2_z0,
    grad_z0) replaced by the notebook's directional operator Axy (σ = E_aniso, default
    aniso_expected) and its magnitude constraint (σ = mag_expected, notebook cell 16).  The dz
    constraints, data rows, σ, TCinv and Ip_c are smooth_fit's (smooth_fit.py:588-627).

    Returns a dict like smooth_fit(return_fit_objects=True) plus 'keep' (Ip_c columns), 'rhs',
    'w' (TCinv diagonal) and 'u' (the direction field)."""
    from .constraint_functions import reference_epoch_keep_cols
    from .smooth_fit import smooth_fit
    E_dz = {k: v for k, v in E_RMS.items() if k not in ('d2z0_dx2', 'dz0_dx', 'z0')}
    S = smooth_fit(data=data, W=W, ctr=ctr, spacing=spacing, E_RMS=E_dz, reference_epoch=reference_epoch,
                   return_fit_objects=True, VERBOSE=False, **kw)
    g = S['grids']['z0']
    if u is None:
        u = circular_field(half_width=max(W['x'], W['y']) / 2)
    if E_aniso is None:
        E_aniso = aniso_expected(E_RMS, g)
    Axy = directional_smoothing_op(g, u)
    Axy.name = 'grad2_z0_aniso'
    Axy.expected = E_aniso + np.zeros(Axy.N_eq)
    mag = lin_op(g, name='mag_z0').one(DOF='z0')
    mag.expected = mag_expected + np.zeros(mag.N_eq)
    Gc = lin_op(None, name='constraints').vstack([Axy, mag, S['Gc']])
    Ec = np.concatenate([Axy.expected, mag.expected, S['Ec']])
    w = 1. / np.concatenate([S['Ed'], Ec])
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], reference_epoch)
    return dict(S, Gc=Gc, Ec=Ec, keep=keep, rhs=rhs, w=w, u=u)
