"""Node-block normals (AᵀA)_bb of lazily formed structured systems (block.hip, round 4): the
class-table kernel k_block_normal_tab (the default when every stencil part has one row scale and
constant coefficients) against the part-descriptor kernel k_block_normal_mf (LSQ_BLK_TAB=0, read at
every call) — the same sums up to the order of the stencil terms, so block-Jacobi CGNR runs the same
iterates: 30 iterations agree to 1e-10 relative, and the converged solves to the stopping rule.
t15: 15 epochs (16-column blocks, the widest dt); ta64: field-valued parts (the table declines:
both calls take the descriptor kernel, bit for bit)."""
import os

import numpy as np
import pytest

from test_gpu_cgnr import _golden_system, _synthetic_system

pytestmark = pytest.mark.gpu


def _run(which, tab, maxit):
    saved = os.environ.get('LSQ_BLK_TAB')
    os.environ['LSQ_BLK_TAB'] = tab
    try:
        if which == 'ta64':   # anisotropic (field-valued) constraint parts
            from lssurf_amd import synthetic
            from lssurf_amd.smooth_fit import FitSystem
            S, _ = synthetic.aniso_system(which)
            fs = FitSystem(S['G_data'], S['Gc'], S['keep'], S['Gc'].col_N, grids=S['grids'])
            w, rhs = S['w'], S['rhs']
        elif which.startswith('t'):
            _, fs, w, rhs = _synthetic_system(which)
        else:
            _, fs, w, rhs = _golden_system(which)
        try:
            fs.solver.set_row_weight(w)
            fs.solver.set_row_mask(np.ones(w.size, bool))
            x, st = fs.solver.solve(rhs, atol=1e-12, btol=1e-12, conlim=1e12, maxit=maxit, precond=3, method=1)
            return x, st
        finally:
            fs.close()
    finally:
        if saved is None:
            os.environ.pop('LSQ_BLK_TAB', None)
        else:
            os.environ['LSQ_BLK_TAB'] = saved


@pytest.mark.parametrize('which', ['sf3d', 't64', 't15', 'ta64'])
def test_block_normal_table_matches_descriptor_kernel(gpu_available, which):
    xa, sa = _run(which, '0', 30)
    xb, sb = _run(which, '1', 30)
    assert sa['method'] == sb['method'] == 1
    rel = np.linalg.norm(xb - xa) / np.linalg.norm(xa)
    if which == 'ta64':
        assert rel == 0.0
    else:
        assert rel <= 1e-10, rel
    xa, sa = _run(which, '0', 0)
    xb, sb = _run(which, '1', 0)
    assert abs(sa['iters'] - sb['iters']) <= 2
    assert np.linalg.norm(xb - xa) / np.linalg.norm(xa) <= 1e-8


def test_block_spanning_nodes_takes_descriptor_kernel(gpu_available):
    """A user block that pairs two (y, x) nodes of one grid (here the z0 columns of x-neighbours,
    coupled by the z0 curvature stencil): the class tables hold only the stencil terms inside one
    node, so the table kernel flags the block and the normals come from the part descriptors —
    the same iterates as LSQ_BLK_TAB=0 (without the flag they silently differed)."""
    def run(tab):
        saved = os.environ.get('LSQ_BLK_TAB')
        os.environ['LSQ_BLK_TAB'] = tab
        try:
            S, fs, w, rhs = _synthetic_system('t64')
            try:
                z0 = np.asarray(S['G_data'].TOC['cols']['z0']).ravel()
                ny, nx = S['grids']['z0'].shape
                pos = np.searchsorted(fs.keep_cols, z0).reshape(ny, nx)
                blocks = [np.array([pos[y, 2 * i], pos[y, 2 * i + 1]]) for y in range(ny) for i in range(nx // 2)]
                fs.solver.set_column_blocks(blocks)
                fs.solver.set_row_weight(w)
                fs.solver.set_row_mask(np.ones(w.size, bool))
                return fs.solver.solve(rhs, atol=1e-12, btol=1e-12, conlim=1e12, maxit=30, precond=3, method=1)
            finally:
                fs.close()
        finally:
            if saved is None:
                os.environ.pop('LSQ_BLK_TAB', None)
            else:
                os.environ['LSQ_BLK_TAB'] = saved

    xa, sa = run('0')
    xb, sb = run('1')
    assert sa['method'] == sb['method'] == 1
    assert np.linalg.norm(xb - xa) / np.linalg.norm(xa) <= 1e-10
