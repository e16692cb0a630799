"""The fused data rows (k_cg_dmf_fused, round 4: t = Ad·p, the x-edge correction and q += Adᵀt in
one launch, td staged in LDS) against the three-kernel path they replace (LSQ_CG_DFUSE=0, read at
every launch): the normal operator q = AᵀA p is equal BIT FOR BIT (the same points summed in the
same order with the same products, the x-edge pass before them), on the golden systems, on grids
with partial tiles (t64: 64 columns, node rows not a multiple of 4), interior and edge tiles (t256),
tiles whose points overflow the LDS staging (tdense: ~10 points per cell), and the solves agree."""
import os

import numpy as np
import pytest

from test_gpu_cgnr import _golden_system, _synthetic_system

pytestmark = pytest.mark.gpu


def _with(flag, fn):
    saved = os.environ.get('LSQ_CG_DFUSE')
    os.environ['LSQ_CG_DFUSE'] = flag
    try:
        return fn()
    finally:
        if saved is None:
            os.environ.pop('LSQ_CG_DFUSE', None)
        else:
            os.environ['LSQ_CG_DFUSE'] = saved


def _system(which):
    if which.startswith('t'):
        _, fs, w, rhs = _synthetic_system(which)
    else:
        _, fs, w, rhs = _golden_system(which)
    return fs, w, rhs


@pytest.mark.parametrize('which', ['sf3d', 'nb_xt', 't64', 't256', 'tdense'])
def test_fused_data_rows_bitwise(gpu_available, which):
    fs, w, rhs = _system(which)
    try:
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.ones(w.size, bool))
        ok, why = fs.solver.cg_available(1)
        assert ok, why
        rng = np.random.default_rng(5)
        p = np.zeros(fs.n_full)
        p[fs.keep_cols] = rng.standard_normal(fs.keep_cols.size)
        qa = _with('0', lambda: fs.solver.normal_apply(p))
        qb = _with('1', lambda: fs.solver.normal_apply(p))
        np.testing.assert_array_equal(qa, qb)
        assert np.count_nonzero(qb) > 0
    finally:
        fs.close()


@pytest.mark.parametrize('which,precond', [('t64', 3), ('t64', 4), ('t256', 4)])
def test_fused_data_rows_solves(gpu_available, which, precond):
    def solve(flag):
        fs, w, rhs = _system(which)
        try:
            fs.solver.set_row_weight(w)
            fs.solver.set_row_mask(np.ones(w.size, bool))
            return _with(flag, lambda: fs.solver.solve(rhs, atol=1e-12, btol=1e-12, conlim=1e12, precond=precond,
                                                      method=1))
        finally:
            fs.close()
    xa, sa = solve('0')
    xb, sb = solve('1')
    assert sa['method'] == sb['method'] == 1
    assert abs(sa['iters'] - sb['iters']) <= 2, (sa['iters'], sb['iters'])
    assert np.linalg.norm(xb - xa) / np.linalg.norm(xa) <= 1e-9
