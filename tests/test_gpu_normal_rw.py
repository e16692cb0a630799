"""GPU parity of the wave-strip normal-stencil operator (k_cg_normal_rw, csrc/lsqr_cg_rw.inc).

By default the library takes it only where its strips are 8 rows or longer (C4, C5); the test
systems are small, so a child process forces it (LSQ_CG_RW=2, read once per process) and checks,
on every system whose stencil the path admits: q = N p equals Aᵀ(A p) of the formed A (the
reference-identical matrix) to 1e-12 on random p, every boundary class included; CGNR with
block-Jacobi and with the multigrid V-cycle (whose level-0 operator is the same kernel) reaches
the golden exact solution (DESIGN.md tolerances).  Systems it does not admit (t15: 15 epochs)
must report the ring kernel and still pass."""
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
for name in ['sf3d', 'nb_xt', 't64', 'tdense', 't256', 't15']:
    if name.startswith('t'):
        D, kw = synthetic.points(name)
        S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
        xs = None
    else:
        g = golden(f'sys_{name}.npz')
        kw = golden_kwargs(g)
        S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
        xs = g['x']
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    w = 1. / np.sqrt((1 / (1. / np.concatenate((S['Ed'], S['Ec'])))) ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    r = {}
    try:
        rng = np.random.default_rng(11)
        dk = rng.random(fs.n_data) > 0.2
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.concatenate([dk, np.ones(fs.n_con, bool)]))
        r['kernel'] = fs.solver.profile_cg(reps=1, precond=3)['normal_kernel']
        A = fs.solver.get_csr()
        err = 0.0
        for _ in range(2):
            pc = rng.standard_normal(A.shape[1])
            pf = np.zeros(fs.n_full)
            pf[fs.keep_cols] = pc
            q = fs.solver.normal_apply(pf)[fs.keep_cols]
            qr = A.T @ (A @ pc)
            err = max(err, float(np.abs(q - qr).max() / np.abs(qr).max()))
        r['op_err'] = err
        if xs is not None:
            for pre in (3, 4):
                ok = fs.solver.cg_available(pre)[0]
                if not ok:
                    continue
                x = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=pre, method=1, **TOL)
                r[f'rel{pre}'] = float(np.linalg.norm(x - xs) / np.linalg.norm(xs))
                r[f'abs{pre}'] = float(np.max(np.abs(x - xs)))
    finally:
        fs.close()
    out[name] = r
json.dump(out, open(sys.argv[2], 'w'))
'''


def test_wave_strip_operator_forced(gpu_available, tmp_path):
    out = tmp_path / 'rw.json'
    env = dict(os.environ, LSQ_CG_RW='2')
    r = subprocess.run([sys.executable, '-c', _CHILD, os.path.dirname(__file__), str(out)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    res = json.load(open(out))
    for name, d in res.items():
        assert d['op_err'] <= 1e-12, (name, d)
        for pre in (3, 4):
            if f'rel{pre}' in d:
                assert d[f'rel{pre}'] <= 1e-6 and d[f'abs{pre}'] <= 1e-4, (name, pre, d)
    for name in ('sf3d', 't64', 'tdense', 't256'):
        assert res[name]['kernel'] == 'wave-strip', (name, res[name])
    assert res['t15']['kernel'] == 'ring', res['t15']   # 15 epochs: outside the path
