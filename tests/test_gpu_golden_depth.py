"""smooth_fit's default solver pinned to the reference at depth, and sigma_extra_keys.

* sys_deep{1,3}.npz (tests/golden/gen_golden.py gen_deep): 48² × 12 nodes, 27 648 unknowns —
  above lsq_dense_max, so smooth_fit's default is CGNR with the multigrid V-cycle on a real
  hierarchy (48 → 25 → 13 → 7 → 4 nodes per side) — run by the reference with the exact dense LS
  oracle at max_iterations 1 and 3 (outliers: the 3-iteration run edits).
* sys_sekeys.npz (gen_sekeys): sigma_extra_keys over two field groups (smooth_fit.py:442-447),
  4 outer iterations.
Tolerances as the other smooth_fit goldens: outputs ≤ 1e-6 relative, ≤ 2 edit
flips (points within rounding of |r/σ| = 3), sigma_extra ≤ 1e-5.
"""
import numpy as np
import pytest

import lssurf_amd as LS
from conftest import golden, golden_kwargs, golden_points

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    ok = np.isfinite(b)
    return np.linalg.norm(a[ok] - b[ok]) / max(np.linalg.norm(b[ok]), 1e-300)


def test_deep_hierarchy_levels(gpu_available):
    """The deep fixture's system really runs a ≥ 4-level multigrid hierarchy."""
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    from lssurf_amd.smooth_fit import FitSystem
    g = golden('sys_deep1.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    assert keep.size == int(g['x'].size) == 27648
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    try:
        assert fs.multigrid_available(np.abs(1. / np.concatenate((S['Ed'], S['Ec']))))
        levels, _ = fs.solver.mg_info()
        assert len(levels) >= 4, levels
    finally:
        fs.close()


@pytest.mark.parametrize('iters', [1, 3])
def test_deep_default_solver_matches_reference(gpu_available, iters):
    g = golden(f'sys_deep{iters}.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), **kw)
    last = S['timing']['lsq_last']
    assert last['method'] == 1 and last['precond'] == 4   # CGNR + multigrid: the default at this size
    tse = S['data'].three_sigma_edit
    flips = int(np.sum(tse != g['data_three_sigma_edit'].astype(bool)))
    assert flips <= 2
    if iters == 1:   # the one solve against the exact LS solution the reference received
        from lssurf_amd.constraint_functions import reference_epoch_keep_cols
        keep = reference_epoch_keep_cols(S['m']['all'].size, S['grids']['dz'], kw['reference_epoch'])
        assert _rel(S['m']['all'][keep], g['x']) < 1e-6
    if flips == 0:
        assert _rel(S['m']['z0'].z0, g['z0']) < 1e-6
        assert _rel(S['m']['dz'].dz, g['dz']) < 1e-6
        assert np.max(np.abs(S['m']['dz'].dz - g['dz'])) < 1e-4
        assert _rel(S['data'].z_est, g['data_z_est']) < 1e-6
        assert _rel(S['data'].sigma_extra, g['data_sigma_extra']) < 1e-5
    for k in ('R_data', 'RMS_data'):
        key = k.split('_', 1)[1]
        store = S['R'] if k.startswith('R_') else S['RMS']
        assert abs(store[key] - float(g[k])) <= 1e-5 * max(abs(float(g[k])), 1e-12), k


def test_sigma_extra_keys_matches_reference(gpu_available):
    g = golden('sys_sekeys.npz')
    kw = golden_kwargs(g)
    assert set(kw['sigma_extra_keys']) == {'low', 'high'}
    S = LS.smooth_fit(data=golden_points(g), **kw)
    tse = S['data'].three_sigma_edit
    flips = int(np.sum(tse != g['data_three_sigma_edit'].astype(bool)))
    assert flips == 0
    se, ref = S['data'].sigma_extra, g['data_sigma_extra']
    sensor = g['in_sensor']
    # two groups, each with its own sigma_extra
    assert np.unique(ref[sensor < 2]).size == 1 and np.unique(ref[sensor >= 2]).size == 1
    assert ref[sensor < 2][0] != ref[sensor >= 2][0]
    assert _rel(se, ref) < 1e-5
    assert _rel(S['m']['z0'].z0, g['z0']) < 1e-6
    assert _rel(S['m']['dz'].dz, g['dz']) < 1e-6
    assert _rel(S['data'].z_est, g['data_z_est']) < 1e-6
