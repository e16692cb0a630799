"""Parity at the BASELINE sizes (C2: 2-D 1024², 500 k points; C3: 512²×12, 1 M points; C4: 1024²×12
grid, 2 M points, 12.6 M unknowns; C5: 2048²×12, 8 M points)
through size-independent properties — the oracle cannot run here, so each property is one the
exact answer must have:
  * the fused normal operator equals Gᵀ(w²∘(G p)) formed through the explicitly assembled CSR
    (lsq_spmv, the lazily formed full G) to 1e-12, and is symmetric;
  * the multigrid, block-Jacobi CGNR and LSQR solutions agree (≤ 1e-7) and each satisfies the
    normal equations: ‖Aᵀ(b − Ax)‖ / (‖A‖₂ ‖b − Ax‖) ≤ 1e-7, Aᵀr through the assembled CSR;
  * the data rows' node gather (lsq_data_colsum, parse_model's count / misfit maps) equals
    G_dataᵀ f through the assembled CSR and is linear."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def c4():
    import lssurf_amd as LS
    from lssurf_amd import synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    from lssurf_amd.smooth_fit import FitSystem
    D, kw = synthetic.points('c4')
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    w = 1. / np.concatenate((S['Ed'], S['Ec']))
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.ones(w.size, bool))
    yield fs, w, rhs
    fs.close()


def _normal_ref(fs, w, pc):
    g = fs.solver.spmv(pc)                 # G p (unweighted, compact columns)
    return fs.solver.spmv(w * w * g, trans=True)


def test_c4_normal_operator_against_assembled_csr(gpu_available, c4):
    fs, w, rhs = c4
    rng = np.random.default_rng(41)
    u = np.zeros(fs.n_full)
    v = np.zeros(fs.n_full)
    u[fs.keep_cols] = rng.standard_normal(fs.keep_cols.size)
    v[fs.keep_cols] = rng.standard_normal(fs.keep_cols.size)
    qu = fs.solver.normal_apply(u)
    qv = fs.solver.normal_apply(v)
    ref = _normal_ref(fs, w, u[fs.keep_cols])
    assert np.linalg.norm(qu[fs.keep_cols] - ref) <= 1e-12 * np.linalg.norm(ref)
    a, b = v @ qu, u @ qv
    assert abs(a - b) <= 1e-12 * (abs(a) + abs(b))
    assert u @ qu > 0


def _anorm2(fs, steps=8):
    """‖A‖₂ by power steps on AᵀA (a lower bound within a few percent after 8 steps)"""
    v = np.zeros(fs.n_full)
    v[fs.keep_cols] = np.random.default_rng(47).standard_normal(fs.keep_cols.size)
    lam = 0.0
    for _ in range(steps):
        v /= np.linalg.norm(v)
        q = fs.solver.normal_apply(v)
        lam = v @ q
        v = q
    return np.sqrt(lam)


def test_c4_solvers_agree_and_satisfy_the_normal_equations(gpu_available, c4):
    fs, w, rhs = c4
    b = w * rhs
    anorm = _anorm2(fs)
    xs = {}
    for name, opts in (('mg', dict(precond=4, method=1)), ('bj', dict(precond=3, method=1)),
                       ('lsqr', dict(precond=3, method=0))):
        x, st = fs.solver.solve(rhs, atol=1e-10, btol=1e-10, conlim=1e8, b_rows=fs.n_data, **opts)
        assert st['istop'] in (1, 2), (name, st)
        xs[name] = x
        r = b - w * fs.solver.spmv(x)
        atr = fs.solver.spmv(w * r, trans=True)
        ratio = np.linalg.norm(atr) / (anorm * np.linalg.norm(r))
        assert ratio <= 1e-7, (name, ratio)   # an iterate 10 % of the way to x* is ~1e-3
    for name in ('bj', 'lsqr'):
        assert np.linalg.norm(xs[name] - xs['mg']) <= 1e-7 * np.linalg.norm(xs['mg']), name


def test_c4_data_colsum_against_assembled_csr(gpu_available, c4):
    fs, w, rhs = c4
    rng = np.random.default_rng(43)
    f = rng.standard_normal(fs.n_data)
    g = rng.standard_normal(fs.n_data)
    cf, cg, cfg = fs.solver.data_colsum(f), fs.solver.data_colsum(g), fs.solver.data_colsum(f + g)
    full = np.zeros(fs.n_data + fs.n_con)
    full[:fs.n_data] = f
    ref = fs.solver.spmv(full, trans=True)          # G_dataᵀ f on the kept columns
    got = cf[fs.keep_cols]
    assert np.linalg.norm(got - ref) <= 1e-12 * np.linalg.norm(ref)
    assert np.linalg.norm(cfg - (cf + cg)) <= 1e-12 * np.linalg.norm(cfg)


@pytest.fixture(scope='module')
def c5a():
    from lssurf_amd import synthetic
    from lssurf_amd.smooth_fit import FitSystem
    S, _ = synthetic.aniso_system('c5a')
    fs = FitSystem(S['G_data'], S['Gc'], S['keep'], S['Gc'].col_N, grids=S['grids'])
    fs.solver.set_row_weight(S['w'])
    fs.solver.set_row_mask(np.ones(S['w'].size, bool))
    yield fs, S['w'], S['rhs']
    fs.close()


def test_c5a_normal_operator_and_solvers(gpu_available, c5a):
    """BASELINE C5 (2048²×12, 8 M points, 50 M unknowns, field-valued anisotropic z0 constraints):
    the normal operator against the assembled CSR, and the multigrid and block-Jacobi solutions
    agreeing and satisfying the normal equations."""
    fs, w, rhs = c5a
    rng = np.random.default_rng(53)
    u = np.zeros(fs.n_full)
    u[fs.keep_cols] = rng.standard_normal(fs.keep_cols.size)
    qu = fs.solver.normal_apply(u)
    ref = _normal_ref(fs, w, u[fs.keep_cols])
    assert np.linalg.norm(qu[fs.keep_cols] - ref) <= 1e-12 * np.linalg.norm(ref)
    anorm = _anorm2(fs)
    b = w * rhs
    xs = {}
    for name, opts in (('mg', dict(precond=4, method=1)), ('bj', dict(precond=3, method=1))):
        x, st = fs.solver.solve(rhs, atol=1e-10, btol=1e-10, conlim=1e8, b_rows=fs.n_data, **opts)
        assert st['istop'] in (1, 2), (name, st)
        xs[name] = x
        r = b - w * fs.solver.spmv(x)
        ratio = np.linalg.norm(fs.solver.spmv(w * r, trans=True)) / (anorm * np.linalg.norm(r))
        assert ratio <= 1e-7, (name, ratio)
    assert np.linalg.norm(xs['bj'] - xs['mg']) <= 1e-7 * np.linalg.norm(xs['mg'])


def _build(config):
    """FitSystem of BASELINE config c2 (2-D z0-only lin_op system) or c3 (smooth_fit 512²×12),
    as bench.py forms it (first-iteration row weights, every row kept)."""
    from lssurf_amd import synthetic
    from lssurf_amd.smooth_fit import FitSystem
    if config in synthetic.CONFIGS_2D:
        G, Gc, grid, w, rhs = synthetic.system2d(config)
        fs = FitSystem(G, Gc, np.arange(G.col_N), G.col_N, grids={'z0': grid})
    else:
        import lssurf_amd as LS
        from lssurf_amd.constraint_functions import reference_epoch_keep_cols
        D, kw = synthetic.points(config)
        S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
        keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
        fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
        w = 1. / np.concatenate((S['Ed'], S['Ec']))
        rhs = np.zeros(w.size)
        rhs[:S['data'].size] = S['data'].z
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.ones(w.size, bool))
    return fs, w, rhs


@pytest.mark.parametrize('config', ['c2', 'c3'])
def test_c2_c3_operator_and_solvers(gpu_available, config):
    """BASELINE C2 and C3 at full size: the normal operator against the assembled CSR (≤ 1e-12)
    and symmetric; every solver smooth_fit / bench.py would use on the system (multigrid where it
    runs, block-Jacobi where there are node blocks, else column scaling; CGNR and LSQR) reaching a
    solution that satisfies the normal equations (≤ 1e-7), the solutions agreeing (≤ 1e-7)."""
    fs, w, rhs = _build(config)
    try:
        rng = np.random.default_rng(59)
        u = np.zeros(fs.n_full)
        v = np.zeros(fs.n_full)
        u[fs.keep_cols] = rng.standard_normal(fs.keep_cols.size)
        v[fs.keep_cols] = rng.standard_normal(fs.keep_cols.size)
        qu, qv = fs.solver.normal_apply(u), fs.solver.normal_apply(v)
        ref = _normal_ref(fs, w, u[fs.keep_cols])
        assert np.linalg.norm(qu[fs.keep_cols] - ref) <= 1e-12 * np.linalg.norm(ref)
        a, b_ = v @ qu, u @ qv
        assert abs(a - b_) <= 1e-12 * (abs(a) + abs(b_))
        anorm = _anorm2(fs)
        b = w * rhs
        pc = 3 if fs.has_blocks else 1
        runs = [('cg', dict(precond=pc, method=1)), ('lsqr', dict(precond=pc, method=0))]
        if fs.solver.cg_available(4)[0]:
            runs.insert(0, ('mg', dict(precond=4, method=1)))
        xs = {}
        for name, opts in runs:
            x, st = fs.solver.solve(rhs, atol=1e-10, btol=1e-10, conlim=1e8, b_rows=fs.n_data, **opts)
            assert st['istop'] in (1, 2), (config, name, st)
            xs[name] = x
            r = b - w * fs.solver.spmv(x)
            ratio = np.linalg.norm(fs.solver.spmv(w * r, trans=True)) / (anorm * np.linalg.norm(r))
            assert ratio <= 1e-7, (config, name, ratio)
        x0 = xs[runs[0][0]]
        for name in xs:
            assert np.linalg.norm(xs[name] - x0) <= 1e-7 * np.linalg.norm(x0), (config, name)
        if config == 'c3':
            assert 'mg' in xs   # the smooth_fit default at this size
    finally:
        fs.close()
