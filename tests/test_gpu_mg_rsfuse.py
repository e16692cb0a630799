"""The restriction fused into the next level's first smoothing step (k_mg_restrict_smooth,
csrc/mg.inc, round 6: MgHier::fuse bit 2, the default LSQ_MG_FUSE=5) against the separate restriction
and smoothing launches (LSQ_MG_FUSE=1; the switch is read at each hierarchy build, but every case runs
in its own child process so nothing else is shared).  The fused kernel computes each coarse
column's right-hand side with the restriction's own order of operations and then the smoother's
XZERO step on it, so the level-0 V-cycle applied to the same vector, the CGNR + multigrid
iteration count and the solution agree to rounding (≤ 1e-12 relative; the run also reports
whether they are bitwise equal), and the solve reaches the golden exact solution (DESIGN.md
tolerances).  Systems: t64, t256 (the BASELINE layout), sf3d_eq_edit and deep1 (the 48²×12 depth
golden, a ≥ 4-level hierarchy).  LSQ_MG_FUSE=13 adds bit 3: on the direct-kernel levels the
operator kernel writes the residual r − N_s x − B x itself (the smoother's MG_RES order) instead of
q, and the separate residual pass is dropped."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_CHILD = r'''
import sys, json
import numpy as np
sys.path.insert(0, sys.argv[1])
import lssurf_amd as LS
from conftest import golden, golden_kwargs, golden_points
from lssurf_amd.constraint_functions import reference_epoch_keep_cols
from lssurf_amd.smooth_fit import FitSystem
from lssurf_amd import synthetic
TOL = dict(atol=1e-12, btol=1e-12, conlim=1e12)
out = {}
for name in ['t64', 't256', 'sf3d_eq_edit', 'deep1']:
    if name.startswith('t'):
        D, kw = synthetic.points(name)
        S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
        xs = None
    else:
        g = golden(f'sys_{name}.npz')
        kw = golden_kwargs(g)
        kw['VERBOSE'] = False
        S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
        xs = g['x']
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    w = np.abs(1. / np.concatenate((S['Ed'], S['Ec'])))
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    r = {}
    try:
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.ones(w.size, bool))
        v = np.zeros(fs.n_full)
        v[fs.keep_cols] = np.random.default_rng(5).standard_normal(fs.keep_cols.size)
        r['V'] = fs.solver.mg_apply(0, 1, v).tolist()
        x = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=4, method=1, **TOL)
        r['iters'] = int(fs.stats['iters'])
        r['x'] = x.tolist()
        if xs is not None:
            r['rel'] = float(np.linalg.norm(x - xs) / np.linalg.norm(xs))
    finally:
        fs.close()
    out[name] = r
json.dump(out, open(sys.argv[2], 'w'))
'''


def _run(tmp_path, tag, env_extra):
    out = tmp_path / f'{tag}.json'
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, '-c', _CHILD, os.path.dirname(__file__), str(out)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.load(open(out))


@pytest.mark.parametrize('fuse', ['5', '13'])
def test_restrict_smooth_fusion_equals_separate_launches(gpu_available, tmp_path, fuse):
    on = _run(tmp_path, 'on', {'LSQ_MG_FUSE': fuse})
    off = _run(tmp_path, 'off', {'LSQ_MG_FUSE': '1'})
    report = {}
    for name in on:
        a, b = on[name], off[name]
        Va, Vb = np.array(a['V']), np.array(b['V'])
        xa, xb = np.array(a['x']), np.array(b['x'])
        report[name] = dict(V_bitwise=bool(np.array_equal(Va, Vb)), x_bitwise=bool(np.array_equal(xa, xb)),
                            iters=(a['iters'], b['iters']))
        assert np.linalg.norm(Va - Vb) <= 1e-12 * np.linalg.norm(Vb), name
        assert a['iters'] == b['iters'], (name, a['iters'], b['iters'])
        assert np.linalg.norm(xa - xb) <= 1e-12 * np.linalg.norm(xb), name
        if 'rel' in a:
            assert a['rel'] <= 1e-6, (name, a['rel'])
    print('rsfuse', fuse, json.dumps(report))
