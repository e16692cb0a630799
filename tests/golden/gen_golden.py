#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/*.npz by running the REFERENCE (SmithB/LSsurf at
/root/reference) in the survey container.

Only this script touches the reference; it is a no-op where /root/reference is absent (the
GPU box).  The reference is imported with the stand-ins of tests/golden/_refstubs.py:
pointCollection containers, and sparseqr.solve/rz = the exact dense LS oracle (oracle/dense.py)
because SuiteSparseQR/PySPQR are unavailable (parity at that boundary rests on uniqueness of the
full-rank LS solution).  Fixtures hold inputs and outputs only — no reference code.

Fixtures
--------
stencils.npz   lin_op triplets (r, c, v, ind0) for every stencil/interp operator on tiny grids
               (lin_op.py:80-309, 163-247), vstack/toCSR of a composite (lin_op.py:555-631,745-753)
sys_*.npz      for each smooth_fit / lin_op configuration: the input points, the exact matrix A
               and rhs b that the reference handed to sparseqr.solve (smooth_fit.py:142), the
               exact LS solution x*, and the smooth_fit outputs (z0, dz, z_est, three_sigma_edit,
               sigma_extra, dzdt_lag1, E sigma grids)
tri.npz        I/O of the reference Cython kernels inv_tr_upper / propagate_qz_errors /
               spsolve_tr_upper on random upper-triangular CSR matrices (incl. overflow)
sys_avg.npz    averaging products (avg_scales, z0_average_scale, avg_masks) and their errors
kat.npz        the analytic amplitude KAT of notebooks/smooth_fit_demo.ipynb cell 8
sys_sekeys.npz sigma_extra_keys: per-group sigma_extra from a data field (smooth_fit.py:442-447)
sys_deep{1,3}.npz a 48²×12 system (27 648 unknowns) deep enough for the multigrid default, lean
sys_aniso*.npz notebooks/smooth_fit_demo_aniso.ipynb's directional-smoothing systems (the notebook's
               own cells 8-10 and 15 executed from the notebook file on the reference LSsurf): the
               2-D notebook system at 41² / 37² and the C5 z0 + dz system at toy size
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

E_RMS_NB = {'d2z0_dx2': 0.03, 'dz0_dx': 75., 'd3z_dx2dt': 0.006, 'd2z_dxdt': 15., 'd2z_dt2': 5000.}


def _csr_arrays(prefix, A):
    A = sp.csr_matrix(A)
    A.sum_duplicates()
    A.sort_indices()
    return {prefix + '_indptr': A.indptr.astype(np.int64), prefix + '_indices': A.indices.astype(np.int32),
            prefix + '_data': A.data, prefix + '_shape': np.array(A.shape)}


def gen_stencils(LS):
    out = {}
    g2 = LS.fd_grid([[0., 400.], [0., 500.]], [100., 100.], name='z0')
    g3 = LS.fd_grid([[0., 300.], [0., 400.], [0., 1.25]], [100., 100., 0.25], name='dz', col_0=30)
    ops = {
        'grad2': LS.lin_op(g2, name='grad2_z0').grad2(DOF='z0'),
        'grad': LS.lin_op(g2, name='grad_z0').grad(DOF='z0'),
        'one': LS.lin_op(g2, name='mag_z0').one(DOF='z0'),
        'grad2_dzdt': LS.lin_op(g3, name='grad2_dzdt').grad2_dzdt(DOF='z', t_lag=1),
        'grad_dzdt': LS.lin_op(g3, name='grad_dzdt').grad_dzdt(DOF='z', t_lag=1),
        'd2z_dt2': LS.lin_op(g3, name='d2z_dt2').d2z_dt2(DOF='z'),
        'dzdt': LS.lin_op(g3, name='dzdt_lag1').dzdt(lag=1),
        'dzdt2': LS.lin_op(g3, name='dzdt_lag2').dzdt(lag=2),
    }
    rng = np.random.default_rng(7)
    y2 = np.r_[rng.uniform(0, 400, 40), 0., 400., 100., 400., 250.]
    x2 = np.r_[rng.uniform(0, 500, 40), 0., 500., 200., 350., 500.]
    out['pts2_y'], out['pts2_x'] = y2, x2
    ops['interp2'] = LS.lin_op(g2, name='interp_z').interp_mtx([y2, x2])
    y3 = np.r_[rng.uniform(0, 300, 40), 0., 300., 100.]
    x3 = np.r_[rng.uniform(0, 400, 40), 0., 400., 200.]
    t3 = np.r_[rng.uniform(0, 1.25, 40), 0., 1.25, 0.5]
    out['pts3_y'], out['pts3_x'], out['pts3_t'] = y3, x3, t3
    ops['interp3'] = LS.lin_op(g3, name='interp_dz').interp_mtx([y3, x3, t3])
    for k, op in ops.items():
        out[k + '_r'] = np.asarray(op.r).ravel()
        out[k + '_c'] = np.asarray(op.c).ravel()
        out[k + '_v'] = np.asarray(op.v).ravel()
        out[k + '_ind0'] = np.asarray(op.ind0).ravel()
        out[k + '_neq'] = np.array(op.N_eq)
    Gc = LS.lin_op(None, name='constraints').vstack([ops['grad2'], ops['grad']])
    out.update(_csr_arrays('vstack', Gc.toCSR()))
    np.savez_compressed(os.path.join(HERE, 'stencils.npz'), **out)


def synth_points(rng, W, ctr, n, with_t=True, outside=0):
    """uniform points in the domain + a few exactly on bounds/nodes + `outside` out-of-bounds."""
    x = ctr['x'] + (rng.random(n) - 0.5) * W['x']
    y = ctr['y'] + (rng.random(n) - 0.5) * W['y']
    t = ctr['t'] + (rng.random(n) - 0.5) * W['t']
    # exact upper/lower bounds and an exact node
    x[:3] = [ctr['x'] + W['x'] / 2, ctr['x'] - W['x'] / 2, ctr['x']]
    y[:3] = [ctr['y'] + W['y'] / 2, ctr['y'], ctr['y'] - W['y'] / 2]
    t[:3] = [ctr['t'] + W['t'] / 2, ctr['t'] - W['t'] / 2, ctr['t']]
    if outside:
        x[3:3 + outside] = ctr['x'] + W['x']          # out of bounds: dropped by smooth_fit
    Lx, Ly = W['x'] / 2, W['y'] / 3
    z = 10 * np.sin(2 * np.pi * x / Lx) * np.cos(2 * np.pi * y / Ly) \
        + 0.5 * t * np.exp(-((x - ctr['x'])**2 + (y - ctr['y'])**2) / (W['x'] / 4)**2) \
        + rng.normal(0, 0.1, n)
    return x, y, t, z


def run_sf(LS, stubs, name, data_dict, sf_kwargs, n_outliers=0, rng=None, extra=None, lean=False):
    """lean: store no matrices (the inputs, the exact first solution x* the oracle returned to
    the reference, and the outputs) — the fixtures of systems too large to commit their A."""
    import pointCollection as pc
    data = pc.data().from_dict(data_dict)
    stubs.CALLS.clear()
    stubs.SOLS.clear()
    S = LS.smooth_fit(data=data, **sf_kwargs)
    out = {'in_' + k: np.asarray(v) for k, v in data_dict.items()}
    A, b = stubs.CALLS[0]
    from oracle import dense
    if lean:
        out['x'] = stubs.SOLS[0]
        out['x_opt'] = np.array(dense.optimality(A, b, stubs.SOLS[0]))
        out['x_shape'] = np.array(A.shape)
    else:
        out.update(_csr_arrays('A', A))
        out['b'] = b
        x = dense.ls_solve_dense(A, b)
        out['x'] = x
        out['x_opt'] = np.array(dense.optimality(A, b, x))
        # last solve (after editing) as well
        A2, b2 = stubs.CALLS[-1]
        out.update(_csr_arrays('Alast', A2))
        out['blast'] = b2
    out['n_solves'] = np.array(len(stubs.CALLS))
    m = S['m']
    out['z0'] = m['z0'].z0
    out['dz'] = m['dz'].dz
    out['m_all'] = m['all']
    d = S['data']
    for f in ['z_est', 'three_sigma_edit', 'sigma_extra']:
        out['data_' + f] = np.asarray(getattr(d, f))
    out['valid_data'] = np.asarray(S['valid_data'])
    for k in m:
        if k.startswith('dzdt_lag'):
            out['m_' + k] = getattr(m[k], k)
    for f in ['count', 'misfit_rms', 'misfit_scaled_rms', 'misfit_notide_rms', 'misfit_notide_scaled_rms']:
        if hasattr(m['z0'], f):   # the notide maps exist when the data carry 'tide' (smooth_fit.py:346-352)
            out['z0_' + f] = getattr(m['z0'], f)
            out['dz_' + f] = getattr(m['dz'], f)
    skip = {'z0', 'dz', 'all', 'extent', 'sensor_bias_grids', 'jitter_bias_grids'}
    for k in m:
        if k not in skip and not k.startswith('dzdt_lag'):     # averaging products
            out['avg_' + k] = np.asarray(getattr(m[k], k))
            area = np.asarray(getattr(m[k], 'cell_area', None))
            if area.dtype != object:
                out['avgarea_' + k] = area
    for k, v in S['R'].items():
        out['R_' + k] = np.array(v)
    for k, v in S['RMS'].items():
        out['RMS_' + k] = np.array(v)
    for k, v in S['E'].items():
        out['E_' + k] = np.asarray(getattr(v, k))
    out['kwargs'] = np.array(repr({k: v for k, v in sf_kwargs.items() if k != 'avg_masks'}))
    if lean:   # the solution-derived grids other fixtures already pin: kept out of the lean file
        out = {k: v for k, v in out.items() if not (k == 'm_all' or k.startswith('m_dzdt') or
                                                      k.startswith('z0_') or k.startswith('dz_'))}
    for k, v in (extra or {}).items():
        out['in_' + k] = np.asarray(v)
    np.savez_compressed(os.path.join(HERE, f'sys_{name}.npz'), **out)
    print(f'{name}: A {A.shape} nnz {A.nnz}, solves {len(stubs.CALLS)}, opt {out["x_opt"]:.2e}')


def gen_systems(LS, stubs):
    rng = np.random.default_rng(20251121)
    # 1. 3-D z0+dz, equal spacing (the C3/C4 structure at toy size)
    W = {'x': 1500., 'y': 1500., 't': 1.25}
    ctr = {'x': 0., 'y': 0., 't': 0.}
    x, y, t, z = synth_points(rng, W, ctr, 700, outside=2)
    run_sf(LS, stubs, 'sf3d', {'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(x.size, 0.1)},
           dict(W=W, ctr=ctr, spacing={'z0': 100., 'dz': 100., 'dt': 0.25}, E_RMS=E_RMS_NB,
                reference_epoch=3, max_iterations=1, VERBOSE=False, dzdt_lags=[1]))
    # 2. finer z0 than dz, 'z0' magnitude constraint, outliers, 3 outer iterations
    W = {'x': 1000., 'y': 800., 't': 1.0}
    x, y, t, z = synth_points(rng, W, ctr, 900)
    bad = rng.random(x.size) > 0.9
    z[bad] += (rng.random(bad.sum()) - 0.5) * 40
    E = dict(E_RMS_NB, z0=50.)
    run_sf(LS, stubs, 'sf3d_edit', {'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(x.size, 0.1)},
           dict(W=W, ctr=ctr, spacing={'z0': 50., 'dz': 100., 'dt': 0.25}, E_RMS=E,
                reference_epoch=2, max_iterations=4, VERBOSE=False, dzdt_lags=[1, 2]))
    # 3. notebooks/smooth_fit_demo.ipynb cell 17 (x-t problem), exactly
    W = {'x': 1.e4, 'y': 200, 't': 2}
    xx = np.arange(-W['x'] / 2, W['x'] / 2, 100)
    amp, lam = 100, 2000
    d0 = {'x': xx, 'y': np.zeros_like(xx), 'z': np.zeros_like(xx), 'time': np.zeros_like(xx) - 0.99,
          'sigma': np.zeros_like(xx) + 1}
    d1 = {'x': xx, 'y': np.zeros_like(xx), 'z': amp - amp * np.cos(2 * np.pi * xx / lam),
          'time': np.zeros_like(xx) + 0.99, 'sigma': np.zeros_like(xx) + 1}
    dd = {k: np.r_[d0[k], d1[k]] for k in d0}
    E = dict(E_RMS_NB)
    run_sf(LS, stubs, 'nb_xt', dd, dict(W=W, ctr=ctr, spacing={'z0': 50, 'dz': 100, 'dt': 0.25},
                                         E_RMS=E, reference_epoch=4, max_iterations=1, VERBOSE=False,
                                         dzdt_lags=[1]))
    # 4. notebook cell 45: reduced-resolution error propagation (compute_E), data gap
    gap = np.abs(dd['x']) > 1000
    dg = {k: v[gap] for k, v in dd.items()}
    run_sf(LS, stubs, 'nb_err', dg, dict(W={'x': 1.e4, 'y': 400, 't': 2}, ctr=ctr,
                                          spacing={'z0': 100, 'dz': 200, 'dt': 0.25}, E_RMS=E,
                                          reference_epoch=4, max_iterations=1, compute_E=True,
                                          VERBOSE=False, dzdt_lags=[1]))


def gen_eq_edit(LS, stubs):
    """Equal z0 / dz spacing (the BASELINE configs' layout) with outliers and 3 outer iterations
    of editing: the structure on which smooth_fit runs the multigrid solver at scale."""
    rng = np.random.default_rng(20251123)
    W = {'x': 1800., 'y': 1500., 't': 1.5}
    ctr = {'x': 0., 'y': 0., 't': 0.}
    x, y, t, z = synth_points(rng, W, ctr, 1200)
    bad = rng.random(x.size) > 0.92
    z[bad] += (rng.random(bad.sum()) - 0.5) * 40
    run_sf(LS, stubs, 'sf3d_eq_edit', {'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(x.size, 0.1)},
           dict(W=W, ctr=ctr, spacing={'z0': 100., 'dz': 100., 'dt': 0.25}, E_RMS=E_RMS_NB,
                reference_epoch=3, max_iterations=3, VERBOSE=False, dzdt_lags=[1]))


def gen_tide(LS, stubs):
    """Data carrying a 'tide' field (parse_model's misfit_notide maps, smooth_fit.py:346-352),
    with outliers and editing so the maps see an edited subset, and sigma_extra_relax."""
    rng = np.random.default_rng(20251124)
    W = {'x': 1200., 'y': 1000., 't': 1.25}
    ctr = {'x': 0., 'y': 0., 't': 0.}
    x, y, t, z = synth_points(rng, W, ctr, 800)
    bad = rng.random(x.size) > 0.9
    z[bad] += (rng.random(bad.sum()) - 0.5) * 40
    tide = 0.3 * np.sin(2 * np.pi * t / 0.5) + rng.normal(0, 0.05, x.size)
    run_sf(LS, stubs, 'tide', {'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(x.size, 0.1), 'tide': tide},
           dict(W=W, ctr=ctr, spacing={'z0': 100., 'dz': 100., 'dt': 0.25}, E_RMS=E_RMS_NB,
                reference_epoch=2, max_iterations=3, VERBOSE=False, dzdt_lags=[1], sigma_extra_relax=True))


def gen_sekeys(LS, stubs):
    """sigma_extra_keys (smooth_fit.py:442-447): two sigma_extra groups built from a data field
    ('sensor' values {0, 1} and {2, 3}, the groups with different extra noise), outliers and 4
    outer iterations, so calc_sigma_extra's per-group RDE (calc_sigma_extra.py:13-44) drives the
    edits."""
    rng = np.random.default_rng(20251125)
    W = {'x': 1400., 'y': 1200., 't': 1.25}
    ctr = {'x': 0., 'y': 0., 't': 0.}
    x, y, t, z = synth_points(rng, W, ctr, 1000)
    sensor = rng.integers(0, 4, x.size).astype(float)
    z = z + np.where(sensor >= 2, rng.normal(0, 0.6, x.size), rng.normal(0, 0.05, x.size))
    bad = rng.random(x.size) > 0.93
    z[bad] += (rng.random(bad.sum()) - 0.5) * 40
    run_sf(LS, stubs, 'sekeys', {'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(x.size, 0.1),
                                 'sensor': sensor},
           dict(W=W, ctr=ctr, spacing={'z0': 100., 'dz': 100., 'dt': 0.25}, E_RMS=E_RMS_NB,
                reference_epoch=2, max_iterations=4, VERBOSE=False, dzdt_lags=[1],
                sigma_extra_keys={'low': {'sensor': [0., 1.]}, 'high': {'sensor': [2., 3.]}}))


def gen_deep(LS, stubs):
    """A system deep enough for smooth_fit's default multigrid solver to run a real hierarchy
    (VERDICT r5 #3a): 48 × 48 (y, x) nodes × 12 epochs, z0 and dz on one 100 m lattice,
    2 points per (y, x) node (C4's density), n = 27 648 unknowns (above lsq_dense_max, so the
    default is CGNR + the V-cycle: 48 → 25 → 13 → 7 → 4 nodes per side).  Run by the reference
    with the exact dense oracle at max_iterations 1 and 3 (outliers: the 3-iteration run edits).
    Lean fixtures: the inputs, the exact first solution and the outputs, no matrices."""
    rng = np.random.default_rng(20251126)
    W = {'x': 4700., 'y': 4700., 't': 2.75}
    ctr = {'x': 0., 'y': 0., 't': 0.}
    x, y, t, z = synth_points(rng, W, ctr, 2 * 48 * 48)
    bad = rng.random(x.size) > 0.95
    z[bad] += (rng.random(bad.sum()) - 0.5) * 40
    for iters in (1, 3):
        run_sf(LS, stubs, f'deep{iters}', {'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(x.size, 0.1)},
               dict(W=W, ctr=ctr, spacing={'z0': 100., 'dz': 100., 'dt': 0.25}, E_RMS=E_RMS_NB,
                    reference_epoch=5, max_iterations=iters, VERBOSE=False, dzdt_lags=[1]), lean=True)


def gen_avg(LS, stubs):
    """Averaging products (grid_functions.py:177-324, lin_op.py:347-488,669-732):
    avg_scales (dz and dz/dt per lag), z0_average_scale and a named avg_masks region, with
    compute_E so their error grids (grid_error) are pinned too."""
    import pointCollection as pc
    rng = np.random.default_rng(20251122)
    W = {'x': 2000., 'y': 2000., 't': 1.25}
    ctr = {'x': 0., 'y': 0., 't': 0.}
    x, y, t, z = synth_points(rng, W, ctr, 1500)
    mx = np.arange(-1000., 1001., 100.)
    my = np.arange(-1000., 1001., 100.)
    mz = ((np.abs(my[:, None] - 200.) < 450.) & (np.abs(mx[None, :] + 100.) < 650.)).astype(float)
    mask = pc.grid.data().from_dict({'x': mx, 'y': my, 'z': mz})
    run_sf(LS, stubs, 'avg', {'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(x.size, 0.1)},
           dict(W=W, ctr=ctr, spacing={'z0': 100., 'dz': 100., 'dt': 0.25}, E_RMS=E_RMS_NB,
                reference_epoch=2, max_iterations=1, VERBOSE=False, dzdt_lags=[1, 2],
                avg_scales=[400., 1000.], z0_average_scale=400., avg_masks={'basin': mask},
                compute_E=True),
           extra={'mask_x': mx, 'mask_y': my, 'mask_z': mz})
    # the same error grids with an EXACT R⁻¹ (the reference's inv_tr_upper drops |x| <= 1e-5):
    # R = chol(AᵀA) of the matrix the reference handed to sparseqr.rz, pushed through the
    # reference's own averaging operators and grid_error
    import scipy.linalg as sla
    from LSsurf.constraint_functions import build_reference_epoch_matrix
    from LSsurf.grid_functions import setup_averaging_ops, setup_avg_mask_ops, setup_z0_avg
    A = stubs.RZ_CALLS[-1]
    R = sla.cholesky((A.T @ A).toarray(), lower=False)
    Rinv = sla.solve_triangular(R, np.eye(R.shape[0]), lower=False)
    kw = dict(W=W, ctr=ctr, spacing={'z0': 100., 'dz': 100., 'dt': 0.25}, E_RMS=E_RMS_NB, reference_epoch=2,
              max_iterations=1, VERBOSE=False, dzdt_lags=[1, 2], avg_scales=[400., 1000.],
              z0_average_scale=400., avg_masks={'basin': mask})
    F = LS.smooth_fit(data=pc.data().from_dict({'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(x.size, 0.1)}),
                      return_fit_objects=True, **kw)
    grids = F['grids']
    Ip_c = build_reference_epoch_matrix(F['G_data'], F['Gc'], grids, 2)
    full = sp.csr_matrix(Ip_c.dot(sp.csr_matrix(Rinv)))
    ops = setup_averaging_ops(grids['dz'], grids['dz'].col_N, kw, grids['dz'].cell_area)
    ops.update(setup_z0_avg(grids, grids['dz'].col_N, kw))
    ops.update(setup_avg_mask_ops(grids['dz'], F['G_data'].col_N, kw['avg_masks'], kw['dzdt_lags']))
    path = os.path.join(HERE, 'sys_avg.npz')
    out = dict(np.load(path, allow_pickle=False))
    for k, op in ops.items():
        out['Eexact_sigma_' + k] = op.grid_error(full)
    np.savez_compressed(path, **out)


def gen_lin2d(LS):
    """2-D z0-only direct system (BASELINE config C2 structure), formed with the reference
    lin_op exactly as notebooks/smooth_fit_demo_aniso.ipynb cell 6 does."""
    rng = np.random.default_rng(20251122)
    g = LS.fd_grid([[0., 2300.], [0., 2300.]], [100., 100.], name='z0')
    n = 300
    y, x = rng.uniform(0, 2300, n), rng.uniform(0, 2300, n)
    z = 10 * np.sin(2 * np.pi * x / 1150) + rng.normal(0, 0.1, n)
    sigma = np.full(n, 0.1)
    G = LS.lin_op(g, name='interp_z').interp_mtx([y, x])
    root = np.sqrt(np.prod(g.delta))
    g2 = LS.lin_op(g, name='grad2_z0').grad2(DOF='z0')
    g2.expected = 0.03 / root * np.ones(g2.N_eq)
    g1 = LS.lin_op(g, name='grad_z0').grad(DOF='z0')
    g1.expected = 75. / root * np.ones(g1.N_eq)
    Gc = LS.lin_op(None, name='constraints').vstack([g2, g1])
    Gcoo = sp.vstack([G.toCSR(), Gc.toCSR()]).tocoo()
    Eall = np.concatenate([sigma, g2.expected, g1.expected])
    rhs = np.concatenate([z, np.zeros(Gc.shape[0])])
    TCinv = sp.dia_matrix((1 / Eall, 0), shape=(rhs.size, rhs.size))
    A = TCinv.dot(Gcoo)
    b = TCinv.dot(rhs)
    from oracle import dense
    xs = dense.ls_solve_dense(A, b)
    out = {'in_x': x, 'in_y': y, 'in_z': z, 'in_sigma': sigma, 'b': b, 'x': xs,
           'x_opt': np.array(dense.optimality(A, b, xs))}
    out.update(_csr_arrays('A', A))
    np.savez_compressed(os.path.join(HERE, 'sys_lin2d.npz'), **out)
    print(f'lin2d: A {A.shape} nnz {A.nnz}, opt {out["x_opt"]:.2e}')


NB_ANISO = '/root/reference/notebooks/smooth_fit_demo_aniso.ipynb'


def _notebook_ns(LS, stubs):
    """Execute the anisotropic notebook's own definitions (cells 8-10: make_system_of_ops,
    scale_op_by_2d_grid, directional_smoothing_op) and its circular direction field (cell 15)
    from the reference notebook file, against the reference LSsurf.  The field's container is
    the stub grid whose interp is pointCollection's bilinear RectBivariateSpline."""
    import json
    import types
    cells = [c for c in json.load(open(NB_ANISO))['cells'] if c['cell_type'] == 'code']
    src = {i: ''.join(c['source']) for i, c in enumerate(cells)}
    need = [k for k, s in src.items() if 'def make_system_of_ops' in s or 'def scale_op_by_2d_grid' in s
            or 'def directional_smoothing_op' in s]
    field = [k for k, s in src.items() if 'velocity field going around in a circle' in s]
    assert len(need) == 3 and len(field) == 1, 'notebook layout changed'
    plt = types.SimpleNamespace(figure=lambda *a, **k: None, quiver=lambda *a, **k: None)
    pcns = types.SimpleNamespace(data=stubs._PcData, grid=types.SimpleNamespace(data=stubs._PcGridRBS))
    ns = {'np': np, 'LSsurf': LS, 'sp': sp, 'pc': pcns, 'plt': plt}
    for k in need + field:
        exec(compile(src[k], f'{NB_ANISO}:cell{k}', 'exec'), ns)
    return ns


def _u_arrays(u, prefix='u'):
    return {prefix + '_x': np.asarray(u.x), prefix + '_y': np.asarray(u.y), prefix + '_u': np.asarray(u.u),
            prefix + '_v': np.asarray(u.v)}


def gen_aniso(LS, stubs):
    """notebooks/smooth_fit_demo_aniso.ipynb (BASELINE C5's constraint), run on the reference:
    (1) the 2-D notebook system of cells 13-18 (directional operator along the circular field,
    E = 0.25, magnitude constraint expected 2) at reduced grid sizes — 41² (every z0 node on a
    field node) with the notebook's eight points, 37² (interpolated field) with seeded points;
    (2) the C5 system at toy size: smooth_fit's z0 + dz system (return_fit_objects) with the z0
    constraints replaced by the directional operator and the magnitude constraint, Ip_c and TCinv
    as smooth_fit.py:613-627 form them.  Each: A, b handed to sparseqr.solve, exact x*."""
    from oracle import dense
    import pointCollection as pc
    ns = _notebook_ns(LS, stubs)
    u = ns['u']
    rng = np.random.default_rng(20251123)
    for n, npts in ((41, 0), (37, 300)):
        g = LS.fd_grid([[-10., 10.], [-10., 10.]], (20. / (n - 1)) * np.ones(2))
        if npts:
            x, y = rng.uniform(-10, 10, npts), rng.uniform(-10, 10, npts)
            z = 10 * np.sin(2 * np.pi * x / 10) * np.cos(2 * np.pi * y / (20 / 3)) + rng.normal(0, 0.1, npts)
        else:   # cell 18
            pts = 5 * np.exp(1j * np.arange(0, 2 * np.pi, np.pi / 4))
            x, y, z = np.real(pts), np.imag(pts), np.ones(pts.shape)
        sigma = 0.1 * np.ones(x.size)
        G_data = LS.lin_op(g, name='interp_z').interp_mtx([y, x])
        Axy = ns['directional_smoothing_op'](g, u)
        Axy.expected = 0.25 + np.zeros(Axy.shape[0])
        mag = LS.lin_op(g, name='mag_z0').one(DOF='z0')
        mag.expected = 2 + np.zeros(mag.N_eq)
        Gc = LS.lin_op(None, name='constraints').vstack([Axy, mag])
        Gcoo = sp.vstack([G_data.toCSR(), Gc.toCSR()]).tocoo()
        E = np.concatenate([sigma, Axy.expected.ravel(), mag.expected.ravel()])
        rhs = np.concatenate([z, np.zeros([Gc.shape[0]])], axis=0)
        TCinv = sp.dia_matrix((1 / E, 0), shape=(rhs.size, rhs.size))
        A, b = TCinv.dot(Gcoo), TCinv.dot(rhs)
        xs = dense.ls_solve_dense(A, b)
        out = {'in_x': x, 'in_y': y, 'in_z': z, 'nodes': np.array(n), 'b': b, 'x': xs,
               'x_opt': np.array(dense.optimality(A, b, xs)), **_u_arrays(u)}
        out.update(_csr_arrays('A', A))
        out.update(_csr_arrays('Axy', Axy.toCSR()))
        np.savez_compressed(os.path.join(HERE, f'sys_aniso{n}.npz'), **out)
        print(f'aniso{n}: A {A.shape} nnz {A.nnz}, opt {out["x_opt"]:.2e}')
    # (2) C5 at toy size
    from LSsurf.constraint_functions import build_reference_epoch_matrix
    W = {'x': 1500., 'y': 1500., 't': 1.25}
    ctr = {'x': 0., 'y': 0., 't': 0.}
    x, y, t, z = synth_points(rng, W, ctr, 900)
    E_dz = {k: v for k, v in E_RMS_NB.items() if k not in ('d2z0_dx2', 'dz0_dx')}
    F = LS.smooth_fit(data=pc.data().from_dict({'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(x.size, 0.1)}),
                      W=W, ctr=ctr, spacing={'z0': 100., 'dz': 100., 'dt': 0.25}, E_RMS=E_dz, reference_epoch=2,
                      return_fit_objects=True, VERBOSE=False)
    grids = F['grids']
    u3 = stubs._PcGridRBS().from_dict({'x': u.x * 75., 'y': u.y * 75., 'u': u.u, 'v': u.v})   # [-750, 750]²
    Axy = ns['directional_smoothing_op'](grids['z0'], u3)
    Axy.expected = E_RMS_NB['d2z0_dx2'] / np.sqrt(np.prod(grids['z0'].delta)) + np.zeros(Axy.shape[0])
    mag = LS.lin_op(grids['z0'], name='mag_z0').one(DOF='z0')
    mag.expected = 2 + np.zeros(mag.N_eq)
    Gc = LS.lin_op(None, name='constraints').vstack([Axy, mag, F['Gc']])
    Ec = np.concatenate([Axy.expected, mag.expected, F['Ec']])
    Ed = F['Ed']
    N_eq = F['G_data'].N_eq + Gc.N_eq
    TCinv = sp.dia_matrix((1. / np.concatenate((Ed, Ec)), 0), shape=(N_eq, N_eq))
    rhs = np.zeros([N_eq])
    rhs[0:F['data'].size] = F['data'].z.ravel()
    Gcoo = sp.vstack([F['G_data'].toCSR(), Gc.toCSR()]).tocoo()
    Ip_c = build_reference_epoch_matrix(F['G_data'], Gc, grids, 2)
    A, b = TCinv.dot(Gcoo.dot(Ip_c)), TCinv.dot(rhs)
    xs = dense.ls_solve_dense(A, b)
    out = {'in_x': x, 'in_y': y, 'in_time': t, 'in_z': z, 'in_sigma': np.full(x.size, 0.1), 'b': b, 'x': xs,
           'x_opt': np.array(dense.optimality(A, b, xs)), 'u_scale': np.array(75.), **_u_arrays(u),
           'kwargs': np.array(repr(dict(W=W, ctr=ctr, spacing={'z0': 100., 'dz': 100., 'dt': 0.25}, E_RMS=E_RMS_NB,
                                         reference_epoch=2)))}
    out.update(_csr_arrays('A', A))
    np.savez_compressed(os.path.join(HERE, 'sys_aniso3d.npz'), **out)
    print(f'aniso3d: A {A.shape} nnz {A.nnz}, opt {out["x_opt"]:.2e}')


def rand_upper(rng, N, density, diag_first=True):
    R = sp.random(N, N, density=density, random_state=rng, format='csr')
    R = sp.triu(R, k=1).tocsr()
    R = R + sp.diags(rng.uniform(1.0, 3.0, N) * np.sign(rng.normal(size=N)))
    R = sp.csr_matrix(R)
    R.sort_indices()
    return R


def gen_tri(LS):
    import importlib
    itu = importlib.import_module('LSsurf.inv_tr_upper').inv_tr_upper
    pqe = importlib.import_module('LSsurf.propagate_qz_errors').propagate_qz_errors
    sst = importlib.import_module('LSsurf.spsolve_tr_upper').spsolve_tr_upper
    rng = np.random.default_rng(99)
    out = {}
    cases = [(1, 1.0), (7, 0.5), (60, 0.08), (250, 0.02)]
    for i, (N, dens) in enumerate(cases):
        R = rand_upper(rng, N, dens)
        out.update(_csr_arrays(f'R{i}', R))
        nnz = max(4, N * N // 4)
        rr, cc, vv, st = itu(R, nnz, 1e-5)
        out[f'inv{i}_rr'], out[f'inv{i}_cc'], out[f'inv{i}_vv'], out[f'inv{i}_st'] = rr, cc, vv, np.array(st)
        out[f'inv{i}_nnz'] = np.array(nnz)
        # a too-small buffer: the overflow/status=1 semantics (smooth_fit.py:240-246 retries)
        small = max(2, N // 2)
        rr, cc, vv, st = itu(R, small, 1e-5)
        out[f'ovf{i}_rr'], out[f'ovf{i}_cc'], out[f'ovf{i}_vv'], out[f'ovf{i}_st'] = rr, cc, vv, np.array(st)
        out[f'ovf{i}_nnz'] = np.array(small)
        out[f'rss{i}'] = pqe(R)
        bb = rng.normal(size=N)
        out[f'b{i}'] = bb
        out[f'sol{i}'] = sst(R, bb)
    out['ncases'] = np.array(len(cases))
    np.savez_compressed(os.path.join(HERE, 'tri.npz'), **out)
    print('tri: ok')


def gen_kat(LS):
    """notebooks/smooth_fit_demo.ipynb cells 4-8: recovered vs analytic sine amplitude."""
    import pointCollection as pc
    W = {'x': 1.e4, 'y': 200, 't': 2}
    ctr = {'x': 0., 'y': 0., 't': 0.}
    spacing = {'z0': 50, 'dz': 100, 'dt': 0.25}
    x = np.arange(-W['x'] / 2, W['x'] / 2, 100)
    lam, amp, sig = 2000, 100, 1
    D = {'x': x, 'y': np.zeros_like(x), 'z': -amp * np.cos(2 * np.pi * x / lam),
         'time': np.zeros_like(x) - 0.5, 'sigma': np.zeros_like(x) + sig}
    dd = {k: np.r_[D[k], D[k]] for k in D}
    dd['time'] = np.r_[D['time'], np.zeros_like(x) + 0.5]
    E_RMS = {'d2z0_dx2': 0.06, 'dz0_dx': 0.06 * 2500, 'd3z_dx2dt': 0.0001, 'd2z_dxdt': 0.0001 * 2500,
             'd2z_dt2': 5000}
    rd = dd['x'].size / W['x'] / W['y']
    Es, Am, Ae = [0.006, 0.001, 0.0003], [], []
    for E in Es:
        E_RMS['d2z0_dx2'] = E
        S = LS.smooth_fit(data=pc.data().from_dict(dd), ctr=ctr, W=W, spacing=spacing, E_RMS=dict(E_RMS),
                          reference_epoch=2, max_iterations=1, VERBOSE=False, dzdt_lags=[1])
        z0 = S['m']['z0']
        row = int(z0.z0.shape[0] / 2)
        Am.append(np.max(np.abs(z0.z0[row, np.abs(z0.x) < 3000])))
        Ae.append(amp / (1 + 16 * E**-2 * np.pi**4 / (lam**4 * rd) * sig**2))
    np.savez_compressed(os.path.join(HERE, 'kat.npz'), E=np.array(Es), A_ref=np.array(Am),
                        A_expected=np.array(Ae), **{'in_' + k: v for k, v in dd.items()})
    print('kat:', Am, Ae)


def main():
    if not os.path.isdir('/root/reference'):
        print('gen_golden: /root/reference absent; keeping committed fixtures')
        return
    import _refstubs
    LS = _refstubs.install()
    sys.modules['LSsurf.smooth_fit'].smooth_fit   # module (LSsurf/__init__.py:6 rebinds the name)
    gens = {'stencils': lambda: gen_stencils(LS), 'tri': lambda: gen_tri(LS), 'lin2d': lambda: gen_lin2d(LS),
            'systems': lambda: gen_systems(LS, _refstubs), 'avg': lambda: gen_avg(LS, _refstubs),
            'kat': lambda: gen_kat(LS), 'aniso': lambda: gen_aniso(LS, _refstubs),
            'eq_edit': lambda: gen_eq_edit(LS, _refstubs), 'tide': lambda: gen_tide(LS, _refstubs),
            'sekeys': lambda: gen_sekeys(LS, _refstubs), 'deep': lambda: gen_deep(LS, _refstubs)}
    for name in (sys.argv[1:] or list(gens)):   # e.g. `gen_golden.py aniso`: only those fixtures
        gens[name]()


if __name__ == '__main__':
    main()
