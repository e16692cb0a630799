"""The anisotropic-constraint system of notebooks/smooth_fit_demo_aniso.ipynb (BASELINE config
C5) at any grid size: a z0 grid on [-10, 10]², data interpolation rows, a directional
second-derivative operator Axy along a circular direction field u (cells 10, 15, 16: d2z/dx2·u²
+ 2·d2z/dxdy·u·v + d2z/dy2·v², E = 0.25) and a magnitude constraint (cell 5, expected 2), handed
to `sparseqr.solve` as TCinv·G, TCinv·rhs (cell 16).  Built with lssurf_amd's lin_op mirror;
points are synthetic: uniform in the domain, z from the §8(d) surface."""
import numpy as np
import scipy.sparse as sp

from . import containers as pc
from .fd_grid import fd_grid
from .lin_op import lin_op


def _scale_op_by_2d_grid(op, data_grid, field, power=None):
    """notebook cell 9: scale each row by `field` interpolated at the row's mean node position."""
    temp = list(np.unravel_index(op.ind0 - op.grid.col_0, op.grid.shape))
    for dim in range(len(temp)):
        temp[dim] = op.grid.bds[dim][0] + op.grid.delta[dim] * temp[dim]
        if temp[dim].ndim > 1:
            temp[dim] = np.mean(temp[dim], axis=1)
    zi = data_grid.interp(temp[1], temp[0], field=field)
    if power is not None:
        zi = zi ** power
    if op.v.ndim == 1:
        op.v *= zi
    else:
        for col in range(op.v.shape[1]):
            op.v[:, col] *= zi
    return op


def _system_of_ops(stencils):
    """notebook cell 8: give every stencil the union of the offsets (zero coefficients added)."""
    offsets = set()
    for st in stencils.values():
        offsets.update(tuple(jj) for jj in zip(*st[0]))
    for st in stencils.values():
        st[1] = list(st[1])
        have = set(tuple(jj) for jj in zip(*st[0]))
        for off in sorted(offsets):
            if off not in have:
                for dim, oo in enumerate(off):
                    st[0][dim].append(oo)
                st[1].append(0)
        st[1] = np.array(st[1])


def directional_smoothing_op(grid, u):
    """notebook cell 10."""
    coeffs = np.array([-1., 2., -1.]) / (grid.delta[0] ** 2)
    stencils = {'d2zdx2': [[[0, 0, 0], [-1, 0, 1]], coeffs],
                'd2zdy2': [[[-1, 0, 1], [0, 0, 0]], coeffs],
                'd2zdxdy': [[[-1, -1, 1, 1], [-1, 1, -1, 1]], np.array([-1., 1., 1., -1]) / (4 * grid.delta[0] ** 2)]}
    _system_of_ops(stencils)
    Axy = lin_op(grid=grid).diff_op(*stencils['d2zdx2'])
    _scale_op_by_2d_grid(Axy, u, 'u', power=2)
    temp = lin_op(grid=grid).diff_op(*stencils['d2zdxdy'])
    _scale_op_by_2d_grid(temp, u, 'v')
    _scale_op_by_2d_grid(temp, u, 'u')
    temp.v *= 2
    Axy.add(temp)
    temp = lin_op(grid=grid).diff_op(*stencils['d2zdy2'])
    _scale_op_by_2d_grid(temp, u, 'v', power=2)
    Axy.add(temp)
    return Axy


def circular_field(step=0.125):
    """notebook cell 15: unit vectors around the origin."""
    xg, yg = np.meshgrid(np.arange(-10, 10.01, step), np.arange(-10, 10.01, step))
    zg = np.abs(xg + 1j * yg)
    vp, up = np.gradient(zg)
    uv = 1j * (up + 1j * vp)
    uv[np.abs(uv) == 0] = 1
    uv /= np.abs(uv)
    return pc.grid.data().from_dict({'x': xg[0, :], 'y': yg[:, 0], 'u': np.real(uv), 'v': np.imag(uv)})


def system(nodes=401, npts=0, seed=20251121 + 5, E_aniso=0.25, mag_expected=2.0):
    """(A, b, grid) with A = TCinv·[G_data; Axy; mag_z0] (COO) and b = TCinv·rhs, as the notebook
    passes them to sparseqr.solve; `nodes` per side on [-10, 10]² (the notebook: 401)."""
    delta = 20. / (nodes - 1)
    g = fd_grid([[-10., 10.], [-10., 10.]], delta * np.ones(2), name='z0')
    rng = np.random.default_rng(seed)
    if npts:
        x, y = rng.uniform(-10, 10, npts), rng.uniform(-10, 10, npts)
        z = 10 * np.sin(2 * np.pi * x / 10) * np.cos(2 * np.pi * y / (20 / 3)) + rng.normal(0, 0.1, npts)
    else:     # the notebook's eight points on a circle (cell 18)
        pts = 5 * np.exp(1j * np.arange(0, 2 * np.pi, np.pi / 4))
        x, y, z = np.real(pts), np.imag(pts), np.ones(pts.size)
    sigma = np.full(x.size, 0.1)
    G_data = lin_op(g, name='interp_z').interp_mtx([y, x])
    Axy = directional_smoothing_op(g, circular_field())
    Axy.expected = E_aniso + np.zeros(Axy.N_eq)
    mag = lin_op(g, name='mag_z0').one(DOF='z0')
    mag.expected = mag_expected + np.zeros(mag.N_eq)
    Gc = lin_op(None, name='constraints').vstack([Axy, mag])
    G = sp.vstack([G_data.toCSR(), Gc.toCSR()]).tocsr()
    E = np.concatenate([sigma, Axy.expected, mag.expected])
    rhs = np.concatenate([z, np.zeros(Gc.N_eq)])
    A = (sp.diags(1. / E) @ G).tocoo()
    return A, rhs / E, g
