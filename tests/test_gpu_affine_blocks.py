"""Node blocks in affine form (lsq_set_column_blocks_affine, round 4): FitSystem hands smooth_fit's
node blocks to the library as (base, stride) per block column and the library forms and checks the
block arrays on the device.  Block-Jacobi and multigrid solves equal the explicit-array path
(lsq_set_column_blocks) bit for bit; a structure that does not hold (wrong full ids, a column in
two blocks, columns left over) is refused and leaves no blocks set."""
import numpy as np
import pytest

from lssurf_amd._native import NativeError
from lssurf_amd.constraint_functions import node_column_blocks, node_column_blocks_affine
from test_gpu_cgnr import _synthetic_system

pytestmark = pytest.mark.gpu

OPTS = dict(atol=1e-12, btol=1e-12, conlim=1e12, method=1)


def _solve(fs, w, rhs, precond):
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.ones(w.size, bool))
    return fs.solver.solve(rhs, precond=precond, **OPTS)


@pytest.mark.parametrize('which', ['t64', 't15'])
@pytest.mark.parametrize('precond', [3, 4])
def test_affine_blocks_equal_explicit_arrays(gpu_available, which, precond):
    S, fs, w, rhs = _synthetic_system(which)
    try:
        assert fs.has_blocks and fs._blocks is None      # the affine path was taken
        xa, sa = _solve(fs, w, rhs, precond)
    finally:
        fs.close()
    S, fs, w, rhs = _synthetic_system(which)
    try:
        fs.solver.set_column_blocks_csr(*node_column_blocks(S['grids'], fs.keep_cols))
        xb, sb = _solve(fs, w, rhs, precond)
    finally:
        fs.close()
    assert sa['iters'] == sb['iters'] and sa['istop'] in (1, 2)
    np.testing.assert_array_equal(xa, xb)


def test_affine_blocks_refused_when_the_structure_does_not_hold(gpu_available):
    S, fs, w, rhs = _synthetic_system('t64')
    try:
        nb, base, stride, fbase, fstride = node_column_blocks_affine(S['grids'], fs.keep_cols)
        bad = [
            (nb, base, stride, fbase + 1, fstride),                      # full ids differ
            (nb, base, np.where(np.arange(base.size) == 1, 0, stride), fbase, fstride),   # shared column
            (nb - 1, base, stride, fbase, fstride),                      # columns left over
            (nb, base + 10 ** 8, stride, fbase, fstride),                # out of range
        ]
        for args in bad:
            with pytest.raises(NativeError):
                fs.solver.set_column_blocks_affine(*args)
        ok, why = fs.solver.cg_available(4)    # nothing left set: no node blocks for the V-cycle
        assert not ok and 'block' in why, why
        fs.solver.set_column_blocks_affine(nb, base, stride, fbase, fstride)
        x, st = _solve(fs, w, rhs, 3)
        assert st['istop'] in (1, 2)
    finally:
        fs.close()
