"""The row-streaming node gather of the matrix-free data rows (k_cg_dmf_atq_rw, round 4) against
the per-node kernel (k_cg_dmf_atq, the default; LSQ_CG_ATQ_RW=0 / 1 read at every launch): q += Adᵀt
sums every node's points in the same order with the same products, so the two are equal BIT FOR
BIT — through lsq_data_colsum (parse_model's count / misfit maps) on random per-point values and
through the normal operator q = AᵀA p, on grids whose node rows are not a multiple of the wave's
row chunk, narrower than a 64-node strip, and with points on the last row / column of nodes."""
import os

import numpy as np
import pytest

from test_gpu_cgnr import _golden_system, _synthetic_system

pytestmark = pytest.mark.gpu


def _both(fn):
    saved = os.environ.get('LSQ_CG_ATQ_RW')
    try:
        os.environ['LSQ_CG_ATQ_RW'] = '0'
        a = fn()
        os.environ['LSQ_CG_ATQ_RW'] = '1'
        b = fn()
    finally:
        if saved is None:
            os.environ.pop('LSQ_CG_ATQ_RW', None)
        else:
            os.environ['LSQ_CG_ATQ_RW'] = saved
    return a, b


@pytest.mark.parametrize('which', ['sf3d', 't64', 't256', 'tdense'])
def test_atq_rw_bitwise_equal(gpu_available, which):
    if which.startswith('t'):
        _, fs, w, rhs = _synthetic_system(which)
    else:
        _, fs, w, rhs = _golden_system(which)
    try:
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.ones(w.size, bool))
        rng = np.random.default_rng(3)
        f = rng.standard_normal(fs.n_data)
        a, b = _both(lambda: fs.solver.data_colsum(f))
        np.testing.assert_array_equal(a, b)
        assert np.count_nonzero(a) > 0
        ok, why = fs.solver.cg_available(1)
        assert ok, why
        p = np.zeros(fs.n_full)
        p[fs.keep_cols] = rng.standard_normal(fs.keep_cols.size)
        qa, qb = _both(lambda: fs.solver.normal_apply(p))
        np.testing.assert_array_equal(qa, qb)
    finally:
        fs.close()
