"""Host mirror (lssurf_amd.fd_grid / lin_op / constraints / smooth_fit formation) against the
reference's own outputs: triplets, ind0 and whole weighted systems must be bit-identical."""
import numpy as np
import pytest
import scipy.sparse as sp

import lssurf_amd as LS
from conftest import SYSTEMS, golden, golden_csr, golden_kwargs, golden_points

STENCILS = {
    'grad2': lambda g2, g3: LS.lin_op(g2, name='grad2_z0').grad2(DOF='z0'),
    'grad': lambda g2, g3: LS.lin_op(g2, name='grad_z0').grad(DOF='z0'),
    'one': lambda g2, g3: LS.lin_op(g2, name='mag_z0').one(DOF='z0'),
    'grad2_dzdt': lambda g2, g3: LS.lin_op(g3, name='grad2_dzdt').grad2_dzdt(DOF='z', t_lag=1),
    'grad_dzdt': lambda g2, g3: LS.lin_op(g3, name='grad_dzdt').grad_dzdt(DOF='z', t_lag=1),
    'd2z_dt2': lambda g2, g3: LS.lin_op(g3, name='d2z_dt2').d2z_dt2(DOF='z'),
    'dzdt': lambda g2, g3: LS.lin_op(g3, name='dzdt_lag1').dzdt(lag=1),
    'dzdt2': lambda g2, g3: LS.lin_op(g3, name='dzdt_lag2').dzdt(lag=2),
}


def _grids():
    g2 = LS.fd_grid([[0., 400.], [0., 500.]], [100., 100.], name='z0')
    g3 = LS.fd_grid([[0., 300.], [0., 400.], [0., 1.25]], [100., 100., 0.25], name='dz', col_0=30)
    return g2, g3


@pytest.mark.parametrize('key', list(STENCILS) + ['interp2', 'interp3'])
def test_lin_op_triplets_bitwise(key):
    d = golden('stencils.npz')
    g2, g3 = _grids()
    if key == 'interp2':
        op = LS.lin_op(g2, name='interp_z').interp_mtx([d['pts2_y'], d['pts2_x']])
    elif key == 'interp3':
        op = LS.lin_op(g3, name='interp_dz').interp_mtx([d['pts3_y'], d['pts3_x'], d['pts3_t']])
    else:
        op = STENCILS[key](g2, g3)
    for attr in ('r', 'c', 'v', 'ind0'):
        np.testing.assert_array_equal(np.ravel(getattr(op, attr)), d[f'{key}_{attr}'], err_msg=attr)
    assert op.N_eq == int(d[f'{key}_neq'])


def test_vstack_tocsr_bitwise():
    d = golden('stencils.npz')
    g2, _ = _grids()
    Gc = LS.lin_op(None, name='constraints').vstack([STENCILS['grad2'](g2, None), STENCILS['grad'](g2, None)])
    A = Gc.toCSR()
    A.sort_indices()
    ref = golden_csr(d, 'vstack')
    np.testing.assert_array_equal(A.indptr, ref.indptr)
    np.testing.assert_array_equal(A.indices, ref.indices)
    np.testing.assert_array_equal(A.data, ref.data)
    assert set(Gc.TOC['rows']) >= {'grad2_z0', 'grad_z0', 'd2z0_dx2', 'dz0_dx', 'constraints'}


def _scipy_formation(S, ref_epoch, in_TSE=None):
    """The reference's formation (smooth_fit.py:613-627, 123-142) on the mirror's lin_ops."""
    G_data, Gc, Ed, Ec = S['G_data'], S['Gc'], S['Ed'], S['Ec']
    N_eq = G_data.N_eq + Gc.N_eq
    Gcoo = sp.vstack([G_data.toCSR(), Gc.toCSR()]).tocoo()
    Gcoo = Gcoo.dot(LS.build_reference_epoch_matrix(G_data, Gc, S['grids'], ref_epoch))
    E_all = 1 / (1. / np.concatenate((Ed, Ec)))
    TC = sp.dia_matrix((1. / np.sqrt(E_all ** 2), 0), shape=(N_eq, N_eq))
    rhs = np.zeros(N_eq)
    rhs[:S['data'].size] = S['data'].z
    A = sp.csr_matrix(TC.dot(Gcoo))
    A.sort_indices()
    return A, TC.dot(rhs)


@pytest.mark.parametrize('name', SYSTEMS)
def test_smooth_fit_system_bitwise(name):
    g = golden(f'sys_{name}.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    A, b = _scipy_formation(S, kw['reference_epoch'])
    ref = golden_csr(g)
    assert A.shape == ref.shape
    np.testing.assert_array_equal(A.indptr, ref.indptr)
    np.testing.assert_array_equal(A.indices, ref.indices)
    np.testing.assert_array_equal(A.data, ref.data)
    np.testing.assert_array_equal(b, g['b'])


def test_operator_structure_records():
    g2, g3 = _grids()
    Gc = LS.lin_op(None, name='constraints').vstack([STENCILS['grad2'](g2, None), STENCILS['grad_dzdt'](None, g3)])
    assert Gc.parts is not None and len(Gc.parts) == 5
    assert [p['row0'] for p in Gc.parts] == sorted(p['row0'] for p in Gc.parts)
    op = LS.lin_op(g3, name='dzdt_lag1').dzdt(lag=1)
    op.normalize_by_unit_product()
    assert op.parts is None


def test_rde_and_sigma_extra():
    rng = np.random.default_rng(0)
    r = rng.normal(0, 2.0, 20000)
    assert abs(LS.RDE(r) - 2.0) < 0.05
    se = LS.calc_sigma_extra(r, np.full(r.size, 1.0), np.ones(r.size, bool))
    assert abs(np.sqrt(1 + se[0] ** 2) - LS.RDE(r)) < 1e-3
    assert np.isnan(LS.RDE(np.array([1.0])))


def test_out_of_scope_options_raise():
    from lssurf_amd import containers as pc
    D = pc.data().from_dict({'x': np.zeros(3), 'y': np.zeros(3), 'time': np.zeros(3), 'z': np.zeros(3),
                             'sigma': np.ones(3)})
    with pytest.raises(NotImplementedError):
        LS.smooth_fit(data=D, W={'x': 1e3, 'y': 1e3, 't': 1}, ctr={'x': 0, 'y': 0, 't': 0},
                      spacing={'z0': 100, 'dz': 100, 'dt': .25}, E_RMS={'d2z0_dx2': 1}, bias_params=['cycle'])


def test_structured_description_of_smooth_fit_system():
    from lssurf_amd import assemble, synthetic
    D, kw = synthetic.points('t64')
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    d = assemble.describe(S['G_data'], S['Gc'])
    assert d is not None
    grids, interp, coords, stencils, npts = d
    assert len(grids) == 2 and interp == [0, 1] and npts == D.size
    assert sum(s.n_eq for s in stencils) == S['Gc'].N_eq
    assert not S['Gc'].materialized          # nothing was built on the host
    # values changed by data -> no structure -> COO path
    op = LS.lin_op(S['grids']['dz'], name='dzdt_lag1').dzdt(lag=1)
    op.normalize_by_unit_product()
    assert op.parts is None


def _same_grid(a, b, rtol):
    a, b = np.asarray(a, float), np.asarray(b, float)
    assert a.shape == b.shape
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    ok = np.isfinite(b)
    np.testing.assert_allclose(a[ok], b[ok], rtol=rtol, atol=rtol * max(np.max(np.abs(b[ok])), 1e-300))


def test_averaging_products_match_reference():
    """avg_scales / z0_average_scale / avg_masks operators applied to the reference's own
    solution reproduce the reference's averaging grids and their cell areas
    (grid_functions.py:177-324, lin_op.py:347-488,669-732)."""
    from conftest import golden_avg_masks
    from lssurf_amd.grid_functions import setup_averaging_ops, setup_avg_mask_ops, setup_grids, setup_z0_avg
    from lssurf_amd.smooth_fit import DEFAULTS
    g = golden('sys_avg.npz')
    args = dict(DEFAULTS)
    args.update(golden_kwargs(g))
    args['avg_masks'] = golden_avg_masks(g)
    grids, _ = setup_grids(args)
    ops = setup_averaging_ops(grids['dz'], grids['dz'].col_N, args, grids['dz'].cell_area)
    ops.update(setup_z0_avg(grids, grids['dz'].col_N, args))
    ops.update(setup_avg_mask_ops(grids['dz'], grids['dz'].col_N, args['avg_masks'], args['dzdt_lags']))
    expect = {k[4:] for k in g.files if k.startswith('avg_')}
    assert expect == {k for k in ops if not k.startswith('dzdt_lag')}
    m0 = g['m_all']
    for k in expect:
        _same_grid(ops[k].grid_prod(m0), g['avg_' + k], 1e-12)
        if 'avgarea_' + k in g.files:
            _same_grid(ops[k].dst_grid.cell_area, g['avgarea_' + k], 1e-12)


def test_sym_range_and_z0_avg_bound():
    """sym_range is symmetric about the centre; a z0 averaging grid whose subscripts reach
    one past the last node raises, as the reference's ravel_multi_index does."""
    from lssurf_amd.grid_functions import setup_grids, setup_z0_avg, sym_range
    from lssurf_amd.smooth_fit import DEFAULTS
    for N, ni, off in [(21, 4, 0.5), (21, 10, 0), (1025, 10, 0.5), (1024, 25, 0)]:
        s = sym_range(N, ni, off)
        assert np.all(np.diff(s) == ni) and s.min() >= 0 and s.max() < N
    args = dict(DEFAULTS, W={'x': 2000., 'y': 2000., 't': 1.}, ctr={'x': 0., 'y': 0., 't': 0.},
                spacing={'z0': 100., 'dz': 100., 'dt': .25}, z0_average_scale=300.)
    grids, _ = setup_grids(args)
    with pytest.raises(ValueError):
        setup_z0_avg(grids, grids['dz'].col_N, args)
