"""Grid set-up for smooth_fit: the column layout of the unknowns and the output products.

Host mirror of LSsurf/grid_functions.py:
  setup_grids           :26-134  z0 (y,x) at col 0, dz (y,x,t) at col N_z0, t grid, cell areas
  calc_cell_area        :169-175 (planar; projected areas need pyproj — see below)
  sum_cell_area         :136-167
  sym_range             :177-185
  setup_z0_avg          :187-207 z0 averaged to z0_average_scale
  setup_averaging_ops   :209-312 dz/dt lag operators, dz and dz/dt averaged over avg_scales
  setup_avg_mask_ops    :314-324 mean dz, dz/dt over named masks
  validate_by_dz_mask   :346-374
"""
import warnings

import numpy as np

from .fd_grid import fd_grid
from .lin_op import lin_op


def setup_grids(args):
    bds = {c: args['ctr'][c] + np.array([-0.5, 0.5]) * args['W'][c] for c in ('x', 'y', 't')}
    if args.get('mask_data') is not None and not isinstance(args['mask_data'], np.ndarray):
        raise NotImplementedError('setup_grids: only ndarray mask_data is supported by lssurf_amd')
    if args.get('mask_file') is not None:
        raise NotImplementedError('setup_grids: mask files are outside lssurf_amd')
    if args.get('lagrangian_coords') is not None:
        raise NotImplementedError('setup_grids: lagrangian grids are outside lssurf_amd')
    mask = args.get('mask_data')
    sp = args['spacing']
    grids = {}
    # a 2-D mask applies to the dz grid only (the reference derives a z0 mask only from dict or
    # time-varying mask objects, grid_functions.py:49-61); lssurf_amd takes it as a bool array on
    # the dz (y, x) nodes
    grids['z0'] = fd_grid([bds['y'], bds['x']], sp['z0'] * np.ones(2), name='z0', srs_proj4=args.get('srs_proj4'))
    grids['dz'] = fd_grid([bds['y'], bds['x'], bds['t']], [sp['dz'], sp['dz'], sp['dt']], name='dz',
                          col_0=grids['z0'].N_nodes, srs_proj4=args.get('srs_proj4'), mask_data=mask,
                          mask_interp_threshold=0.95)
    grids['t'] = fd_grid([bds['t']], [sp['dt']], name='t')
    grids['z0'].cell_area = calc_cell_area(grids['z0'])
    if np.any(grids['dz'].delta[0:2] >= grids['z0'].delta):
        grids['dz'].cell_area = sum_cell_area(grids['z0'], grids['dz'])
    else:
        grids['dz'].cell_area = calc_cell_area(grids['dz'])
        if grids['dz'].mask is not None:
            grids['dz'].cell_area = grids['dz'].cell_area * grids['dz'].mask
    if grids['z0'].mask is not None:
        grids['z0'].cell_area = grids['z0'].cell_area * grids['z0'].mask
    return grids, bds


def calc_cell_area(grid):
    if grid.srs_proj4 is not None:
        warnings.warn('calc_cell_area: projected (srs_proj4) cell areas need pyproj; using planar areas')
    return np.ones(grid.shape[0:2]) * grid.delta[0] * grid.delta[1]


def sum_cell_area(grid_f, grid_c, cell_area_f=None, return_op=False, sub0s=None, taper=True):
    if cell_area_f is None:
        cell_area_f = calc_cell_area(grid_f) * grid_f.mask
    dims = [0, 1, 2] if cell_area_f.ndim == 3 else [0, 1]
    if not return_op:
        try:
            if np.all(grid_f.ctrs[0] == grid_c.ctrs[0]) and np.all(grid_f.ctrs[1] == grid_c.ctrs[1]):
                return cell_area_f.copy()
        except ValueError:
            pass
    n_k = (grid_c.delta[0:2] / grid_f.delta[0:2] + 1).astype(int)
    if len(dims) == 3:
        n_k = np.array(list(n_k) + [1])
    fine = fd_grid([grid_f.bds[d] for d in dims], deltas=grid_f.delta[dims])
    op = lin_op(grid=fine).sum_to_grid3(n_k, sub0s=sub0s, taper=True, valid_equations_only=False, dims=dims)
    result = op.toCSR().dot(cell_area_f.ravel()).reshape(grid_c.shape[dims])
    return (result, op) if return_op else result


def sym_range(N, ni, offset=0.5):
    """Centre subscripts of averaging cells of ni nodes, symmetric about the grid centre
    (grid_functions.py:177-185)."""
    out = np.arange(ni * offset, N / 2, ni)
    if offset == 0:
        out = np.r_[-out[-1:0:-1], out] + int(np.floor(N / 2))
    else:
        out = np.r_[-out[-1::-1], out] + int(np.floor(N / 2))
    return np.floor(out[np.abs(out - N / 2) <= N / 2 - ni / 2]).astype(int)


def setup_averaging_ops(grid, col_N, args, cell_area=None):
    """dz/dt at each lag, and dz and dz/dt averaged over ``avg_scales`` (grid_functions.py:209-312).
    Only the 2-D-mask branches: 3-D (time-varying) masks are outside lssurf_amd."""
    ops = {}
    if args.get('dzdt_lags') is not None:
        if grid.mask_3d is not None:
            raise NotImplementedError('setup_averaging_ops: 3-D masks are outside lssurf_amd')
        for lag in args['dzdt_lags']:
            name = 'dzdt_lag' + str(lag)
            op = lin_op(grid, name=name, col_N=col_N).dzdt(lag=lag).ravel()
            op.dst_grid.cell_area = grid.cell_area
            op.normalize_by_unit_product()
            ops[name] = op
    if args.get('avg_scales') is None or args.get('dzdt_lags') is None:
        return ops
    n_grid = [c.size for c in grid.ctrs]
    for scale in args['avg_scales']:
        name = 'avg_dz_' + str(int(scale)) + 'm'
        kernel_N = np.floor(np.array([scale / d for d in grid.delta[0:2]] + [1])).astype(int)
        # the largest scale is centred on the grid centre, the others on odd multiples of δ
        offset = 0 if scale == np.max(args['avg_scales']) else 0.5
        sub0s = np.meshgrid(sym_range(n_grid[0], kernel_N[0], offset=offset),
                            sym_range(n_grid[1], kernel_N[1], offset=offset),
                            np.arange(grid.shape[2], dtype=int), indexing='ij')
        op = lin_op(grid, name=name, col_N=col_N).sum_to_grid3(kernel_N + 1, sub0s=sub0s, taper=True)
        op.apply_mask(mask=cell_area)
        if cell_area is not None:
            op.normalize_by_unit_product()
        else:
            op.v /= (kernel_N[0] * kernel_N[1])
        op.dst_grid.cell_area = sum_cell_area(grid, op.dst_grid, sub0s=sub0s, cell_area_f=cell_area)
        ops[name] = op
        for lag in args['dzdt_lags']:
            dz_name = 'avg_dzdt_' + str(int(scale)) + 'm' + '_lag' + str(lag)
            op = lin_op(grid, name=name, col_N=col_N)
            op.sum_to_grid3(kernel_N + 1, sub0s=sub0s, lag=lag, taper=True).apply_2d_mask(mask=cell_area)
            if cell_area is not None:
                # expected number of nonzero entries per node times the per-epoch weight
                op.normalize_by_unit_product(wt=2 / (lag * grid.delta[2]))
            else:
                op.v /= (kernel_N[0] * kernel_N[1])
            ops[dz_name] = op
    return ops


def setup_z0_avg(grids, col_N, args):
    """z0 averaged to ``z0_average_scale`` (grid_functions.py:187-207)."""
    if args.get('z0_average_scale') is None:
        return {}
    scale = args['z0_average_scale']
    name = 'avg_z0_' + str(int(scale)) + 'm'
    g = grids['z0']
    kernel_N = np.floor(np.array([scale / d for d in g.delta[0:2]])).astype(int)
    n_grid = [c.size for c in g.ctrs]
    sub0s = np.meshgrid(*[np.arange(0, n_grid[d] + 1, kernel_N[d]) for d in (0, 1)], indexing='ij')
    op = lin_op(g, name=name, col_N=col_N).sum_to_grid3(kernel_N + 1, sub0s=sub0s, taper=True,
                                                       valid_equations_only=False)
    op.apply_mask(g.cell_area)
    op.normalize_by_unit_product()
    return {name: op}


def setup_avg_mask_ops(grid, col_N, avg_masks, dzdt_lags):
    """Mean dz (and dz/dt per lag) over named 2-D masks (grid_functions.py:314-324)."""
    if avg_masks is None:
        return {}
    ops = {}
    for name, mask in avg_masks.items():
        ops[name + '_avg_dz'] = lin_op(grid, col_N=col_N, name=name + '_avg_dz').mean_of_mask(mask, dzdt_lag=None)
        for lag in dzdt_lags:
            key = name + f'_avg_dzdt_lag{lag}'
            ops[key] = lin_op(grid, col_N=col_N, name=key).mean_of_mask(mask, dzdt_lag=lag)
    return ops


def validate_by_dz_mask(data, grids, valid_data):
    dz = grids['dz']
    if dz.mask_3d is not None:
        tmp = dz.copy()
        tmp.col_0, tmp.col_N = 0, np.prod(tmp.shape)
        sampled = lin_op(tmp, name='interp_z').interp_mtx(data.coords()).toCSR().dot(
            dz.mask_3d.ravel().astype(float))
    else:
        flat = np.ravel(dz.mask).astype(float)
        if flat.size and np.all(flat == flat[0]) and np.isfinite(flat[0]) and flat[0] in (0.0, 1.0):
            # uniform 0/1 mask: the bilinear weights sum to 1, so every point samples the mask
            # value itself (the threshold below decides the same way without forming the operator)
            pts = data.coords()[0:2]
            sampled = np.full(np.size(pts[0]), flat[0])
        else:
            tmp = fd_grid(dz.bds[0:2], dz.delta[0:2])
            sampled = lin_op(tmp, name='interp_z').interp_mtx(data.coords()[0:2]).toCSR().dot(flat)
    sampled[~np.isfinite(sampled)] = 0
    good = sampled > 0.5
    if np.any(~good):
        data.index(good)
        valid_data[valid_data] = good
