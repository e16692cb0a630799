"""GPU parity of the multigrid preconditioner (lsq_opts.precond = 4; lssurf_amd/csrc/mg.inc).

* every level operator equals the host (scipy) hierarchy built from the formed A: Galerkin
  PᵀN_sP of the stencil rows + the (y, x)-lumped data rows (tests/mg_host.py), ≤ 1e-11 relative;
* the V-cycle is a symmetric positive-definite operator (a valid PCG preconditioner);
* PCG with it reaches the exact LS solution within DESIGN.md's tolerance (‖x−x*‖/‖x*‖ ≤ 1e-6,
  max|x−x*| ≤ 1e-4 m), and in far fewer iterations than block-Jacobi."""
import numpy as np
import pytest

from conftest import golden
from mg_host import hierarchy
from test_gpu_cgnr import REL, ABS, TOL, _golden_system, _synthetic_system

pytestmark = pytest.mark.gpu


def _prepare(fs, w, keep):
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.concatenate([keep, np.ones(fs.n_con, bool)]))
    ok, why = fs.solver.cg_available(4)
    assert ok, why


@pytest.mark.parametrize('which', ['t64', 't15', 'tdense'])
def test_mg_level_operators_match_host_galerkin(gpu_available, which):
    S, fs, w, rhs = _synthetic_system(which)
    rng = np.random.default_rng(11)
    keep = rng.random(fs.n_data) > 0.15          # edited data rows, as the outer loop sets
    try:
        _prepare(fs, w, keep)
        levels, tref = fs.solver.mg_info()
        A = fs.solver.get_csr()
        ny, nx, nt = S['grids']['dz'].shape
        host = hierarchy(A, int(keep.sum()), fs.keep_cols, ny, nx, nt)
        assert len(host) == len(levels), (len(host), levels)
        for l, ((shape, kmask, N), (S0, S1, nf)) in enumerate(zip(host, levels)):
            assert shape == (S0, S1) and nf == kmask.size
            if l == len(levels) - 1:
                break                                # coarsest: dense inverse, no operator kernel
            for _ in range(2):
                x = np.where(kmask, rng.standard_normal(nf), 0.0)
                y = fs.solver.mg_apply(l, 0, x)
                yr = N @ x
                err = np.abs(y - yr).max() / np.abs(yr).max()
                assert err <= 1e-11, (l, err)
                assert np.all(y[~kmask] == 0.0)
            lam = fs.solver.mg_apply(l, 2)
            assert np.isfinite(lam) and lam > 0.5, (l, lam)
    finally:
        fs.close()


@pytest.mark.parametrize('kt', ['0', '1', '2'])
def test_mg_tile_kernels_match_host_galerkin(gpu_available, kt):
    """t256: levels 1 and 2 (129² and 65² nodes × 13 columns) run the coarse tile kernel — k_mg_tile
    (LSQ_MG_TILE_KT=0), or the class-compressed k_mg_tile_kt with scalar (1) or LDS-staged (2, the
    default) coefficients; every variant's level operator equals the host Galerkin product."""
    import os
    saved = os.environ.get('LSQ_MG_TILE_KT')
    os.environ['LSQ_MG_TILE_KT'] = kt
    S, fs, w, rhs = _synthetic_system('t256')
    rng = np.random.default_rng(12)
    keep = rng.random(fs.n_data) > 0.15
    try:
        _prepare(fs, w, keep)
        levels, tref = fs.solver.mg_info()
        A = fs.solver.get_csr()
        ny, nx, nt = S['grids']['dz'].shape
        host = hierarchy(A, int(keep.sum()), fs.keep_cols, ny, nx, nt)
        assert len(host) == len(levels), (len(host), levels)
        for l in (1, 2):
            (shape, kmask, N), (S0, S1, nf) = host[l], levels[l]
            assert shape == (S0, S1)
            if l == 1:
                assert nf > 1 << 16   # tiled (MG_TILE_MIN)
            x = np.where(kmask, rng.standard_normal(nf), 0.0)
            y = fs.solver.mg_apply(l, 0, x)
            yr = N @ x
            err = np.abs(y - yr).max() / np.abs(yr).max()
            assert err <= 1e-11, (l, err)
            assert np.all(y[~kmask] == 0.0)
    finally:
        fs.close()
        if saved is None:
            os.environ.pop('LSQ_MG_TILE_KT', None)
        else:
            os.environ['LSQ_MG_TILE_KT'] = saved


def test_mg_vcycle_is_spd(gpu_available):
    S, fs, w, rhs = _synthetic_system('t64')
    rng = np.random.default_rng(5)
    try:
        _prepare(fs, w, np.ones(fs.n_data, bool))
        nf = fs.n_full
        kmask = np.zeros(nf, bool)
        kmask[fs.keep_cols] = True
        u = np.where(kmask, rng.standard_normal(nf), 0.0)
        v = np.where(kmask, rng.standard_normal(nf), 0.0)
        Vu, Vv = fs.solver.mg_apply(0, 1, u), fs.solver.mg_apply(0, 1, v)
        Vu2 = fs.solver.mg_apply(0, 1, u)
    finally:
        fs.close()
    assert np.array_equal(Vu, Vu2)                   # deterministic
    assert np.all(Vu[~kmask] == 0.0)
    a, b = v @ Vu, u @ Vv
    assert abs(a - b) <= 1e-10 * (abs(a) + abs(b)), (a, b)
    assert u @ Vu > 0 and v @ Vv > 0


@pytest.mark.parametrize('name', ['sf3d', 'sf3d_eq_edit', 'sf3d_edit', 'nb_xt', 'nb_err'])
def test_mg_pcg_matches_exact_solution(gpu_available, name):
    """sf3d: z0 and dz on one lattice; sf3d_edit / nb_xt / nb_err: z0 on a 2× refinement of the dz
    lattice (the notebooks' z0 50 m / dz 100 m) — the hierarchy starts with the z0-refined level."""
    g, fs, w, rhs = _golden_system(name)
    try:
        ok, why = fs.solver.cg_available(4)
        assert ok, why
        x = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=4, method=1, maxit=5000, **TOL)
        st = fs.stats
    finally:
        fs.close()
    xs = g['x']
    assert st['method'] == 1 and st['istop'] in (1, 2), st
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) <= REL
    assert np.max(np.abs(x - xs)) <= ABS


@pytest.mark.parametrize('which', ['t64', 't256'])
def test_mg_pcg_iterations_and_solution(gpu_available, which):
    """Same solution as block-Jacobi CGNR (and LSQR) in a fraction of the iterations; masked rows,
    re-weighting and a warm start included."""
    S, fs, w, rhs = _synthetic_system(which)
    rng = np.random.default_rng(2)
    keep = rng.random(fs.n_data) > 0.1
    w2 = w * np.where(np.arange(w.size) < fs.n_data, rng.uniform(0.5, 2, w.size), 1.0)
    try:
        xb = fs.solve(w2, keep, rhs, precond=3, method=1, **TOL)
        it_bj = fs.stats['iters']
        xm = fs.solve(w2, keep, rhs, precond=4, method=1, **TOL)
        st = dict(fs.stats)
        xw = fs.solve(w2, keep, rhs, x0=xm * (1 + 1e-4), precond=4, method=1, **TOL)
        it_warm = fs.stats['iters']
    finally:
        fs.close()
    assert st['method'] == 1 and st['istop'] in (1, 2), st
    assert np.linalg.norm(xm - xb) / np.linalg.norm(xb) <= 1e-8
    assert np.linalg.norm(xw - xb) / np.linalg.norm(xb) <= 1e-8
    assert st['iters'] * 5 <= it_bj, (st['iters'], it_bj)
    assert it_warm <= st['iters']


def test_mg_stiff(gpu_available):
    """Stiff E_RMS (SURVEY.md §8(d) stress variant): the V-cycle stays a good preconditioner."""
    S, fs, w, rhs = _synthetic_system(stiff=True)
    keep = np.ones(fs.n_data, bool)
    try:
        xl = fs.solve(w, keep, rhs, precond=3, method=1, **TOL)
        it_bj = fs.stats['iters']
        xm = fs.solve(w, keep, rhs, precond=4, method=1, **TOL)
        st = fs.stats
    finally:
        fs.close()
    assert st['method'] == 1 and st['istop'] in (1, 2), st
    assert np.linalg.norm(xm - xl) / np.linalg.norm(xl) <= 1e-7
    assert st['iters'] * 3 <= it_bj, (st['iters'], it_bj)


def test_mg_rejects_lsqr_and_unstructured(gpu_available):
    from lssurf_amd._native import NativeError
    S, fs, w, rhs = _synthetic_system('t64')
    try:
        with pytest.raises(NativeError):
            fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=4, method=0, **TOL)
    finally:
        fs.close()


def test_smooth_fit_multigrid_default(gpu_available):
    """smooth_fit's 'auto' preconditioner picks the multigrid V-cycle above lsq_dense_max (forced
    here with lsq_dense_max=0) and its outputs match the reference's golden fit."""
    from conftest import golden_kwargs, golden_points
    import lssurf_amd as LS
    g = golden('sys_sf3d.npz')
    out = LS.smooth_fit(data=golden_points(g), lsq_dense_max=0, **golden_kwargs(g))
    assert out['timing']['lsq_last']['method'] == 1
    for got, ref in ((out['m']['z0'].z0, g['z0']), (out['m']['dz'].dz, g['dz']), (out['data'].z_est, g['data_z_est'])):
        ok = np.isfinite(ref)
        assert np.linalg.norm(got[ok] - ref[ok]) / np.linalg.norm(ref[ok]) < 1e-6
    assert np.nanmax(np.abs(out['m']['dz'].dz - g['dz'])) < ABS
    assert np.array_equal(out['data'].three_sigma_edit, g['data_three_sigma_edit'])


def _mixed_system(which):
    if which == 't64z':
        S, fs, w, rhs = _synthetic_system('t64z')
    else:
        g, fs, w, rhs = _golden_system(which)
    return fs, w, rhs


@pytest.mark.parametrize('which', ['t64z', 'nb_xt', 'sf3d_edit'])
def test_mg_z0_refined_operator_and_vcycle(gpu_available, which):
    """z0 on a 2× refinement of the dz lattice: the fine level's operator equals AᵀA of the formed
    A (≤ 1e-12), the hierarchy below is the dz lattice's (level 1: the dz lattice), and the
    V-cycle is symmetric positive definite."""
    fs, w, rhs = _mixed_system(which)
    rng = np.random.default_rng(9)
    keep = rng.random(fs.n_data) > 0.1
    try:
        _prepare(fs, w, keep)
        levels, tref = fs.solver.mg_info()
        assert levels[0][2] == fs.n_full and levels[1][0] == (levels[0][0] + 1) // 2
        A = fs.solver.get_csr()
        nf = fs.n_full
        kmask = np.zeros(nf, bool)
        kmask[fs.keep_cols] = True
        x = np.where(kmask, rng.standard_normal(nf), 0.0)
        y = fs.solver.mg_apply(0, 0, x)[fs.keep_cols]
        yr = A.T @ (A @ x[fs.keep_cols])
        assert np.abs(y - yr).max() <= 1e-12 * np.abs(yr).max()
        assert fs.solver.mg_apply(0, 2) > 0.5
        u = np.where(kmask, rng.standard_normal(nf), 0.0)
        v = np.where(kmask, rng.standard_normal(nf), 0.0)
        Vu, Vv = fs.solver.mg_apply(0, 1, u), fs.solver.mg_apply(0, 1, v)
    finally:
        fs.close()
    assert np.all(Vu[~kmask] == 0.0)
    a, b = v @ Vu, u @ Vv
    assert abs(a - b) <= 1e-10 * (abs(a) + abs(b)), (a, b)
    assert u @ Vu > 0 and v @ Vv > 0


def test_mg_z0_refined_iterations(gpu_available):
    """t64z (z0 127², dz 64² × 12): multigrid and block-Jacobi CGNR reach the same solution, the
    V-cycle in a fraction of the iterations; edited rows and re-weighting included."""
    fs, w, rhs = _mixed_system('t64z')
    rng = np.random.default_rng(4)
    keep = rng.random(fs.n_data) > 0.1
    w2 = w * np.where(np.arange(w.size) < fs.n_data, rng.uniform(0.5, 2, w.size), 1.0)
    try:
        xb = fs.solve(w2, keep, rhs, precond=3, method=1, **TOL)
        it_bj = fs.stats['iters']
        xm = fs.solve(w2, keep, rhs, precond=4, method=1, **TOL)
        st = dict(fs.stats)
    finally:
        fs.close()
    assert st['method'] == 1 and st['istop'] in (1, 2), st
    assert np.linalg.norm(xm - xb) / np.linalg.norm(xb) <= 1e-8
    assert st['iters'] * 4 <= it_bj, (st['iters'], it_bj)


_PERSIST_CHILD = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from test_gpu_cgnr import _synthetic_system, TOL
S, fs, w, rhs = _synthetic_system('t64')
try:
    x = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=4, method=1, **TOL)
    np.save(sys.argv[2], np.concatenate([[fs.stats['iters']], x]))
finally:
    fs.close()
'''


def test_mg_persistent_coarse_levels(gpu_available, tmp_path):
    """k_mg_coarse (the small coarse levels in one persistent launch with grid barriers; off by
    default, LSQ_MG_PERSIST) gives the launch-per-kernel V-cycle's solve: run in a child process
    with it on (t64: levels 33², 17², 9²), compared with this process's default."""
    import os
    import subprocess
    import sys
    out = tmp_path / 'x.npy'
    env = dict(os.environ, LSQ_MG_PERSIST='16384', LSQ_MG_PWG='32')
    r = subprocess.run([sys.executable, '-c', _PERSIST_CHILD, os.path.dirname(__file__), str(out)], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.load(out)
    S, fs, w, rhs = _synthetic_system('t64')
    try:
        x = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=4, method=1, **TOL)
        it = fs.stats['iters']
    finally:
        fs.close()
    assert abs(int(got[0]) - it) <= 1, (got[0], it)
    assert np.linalg.norm(got[1:] - x) <= 1e-8 * np.linalg.norm(x)


_POW_CHILD = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from test_gpu_cgnr import _synthetic_system, TOL
S, fs, w, rhs = _synthetic_system(sys.argv[3])
try:
    x = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=4, method=1, **TOL)
    levels, _ = fs.solver.mg_info()
    lam = [fs.solver.mg_apply(l, 2) for l in range(len(levels) - 1)]
    np.save(sys.argv[2], np.concatenate([[fs.stats['iters']], lam, x]))
finally:
    fs.close()
'''


@pytest.mark.parametrize('which', ['t64', 't256'])
def test_mg_concurrent_power_steps_match_serial(gpu_available, tmp_path, which):
    """The per-solve set-up runs the coarse levels' power steps on a second stream pair beside
    level 0's (each level its own vectors, scalars and partials): λ of every level and the solve
    equal, bit for bit, a child process that runs them in turn (LSQ_MG_POW_CONC=0)."""
    import os
    import subprocess
    import sys
    got = {}
    for conc in ('0', '1'):
        out = tmp_path / f'x{conc}.npy'
        env = dict(os.environ, LSQ_MG_POW_CONC=conc)
        r = subprocess.run([sys.executable, '-c', _POW_CHILD, os.path.dirname(__file__), str(out), which], env=env,
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        got[conc] = np.load(out)
    np.testing.assert_array_equal(got['0'], got['1'])

