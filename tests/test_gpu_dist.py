"""GPU parity of the multi-GPU solve (lssurf_amd.dist through liblsqsurf's C ABI).

The y-slab distributed LSQR runs the same recurrence as the single-GPU solve; only the order
of the floating-point sums in the inner products differs (per-rank partials, then the
all-reduce), so the iterates agree to rounding and the converged solutions to the solver
tolerance: ||x_dist - x_1gpu|| / ||x_1gpu|| <= 1e-8 at atol = btol = 1e-12, and the distributed
solution meets the parity bar against the exact LS solution (1e-6 relative) on the golden
system.  Virtual ranks (all ranks in this process) exercise the partition, halo plans and
exchange order on one GPU; a one-rank RCCL communicator exercises the RCCL transport."""
import socket

import numpy as np
import pytest

import lssurf_amd as LS
from conftest import golden, golden_kwargs, golden_points
from lssurf_amd import dist, synthetic
from lssurf_amd.constraint_functions import reference_epoch_keep_cols
from lssurf_amd.smooth_fit import FitSystem

pytestmark = pytest.mark.gpu
TOL = dict(atol=1e-12, btol=1e-12, conlim=1e12, precond=1)


def _problem(S, kw):
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    E_all = 1 / (1. / np.concatenate((S['Ed'], S['Ec'])))
    w = 1. / np.sqrt(E_all ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    return keep, w, rhs


def _t64():
    D, kw = synthetic.points('t64')
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    return S, kw


def _single(S, keep, w, rhs):
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N)
    x = fs.solve(w, np.ones(fs.n_data, bool), rhs, **TOL)
    st = fs.stats
    fs.close()
    return x, st


@pytest.mark.parametrize('structured', [True, False])
@pytest.mark.parametrize('nranks', [2, 3, 4])
def test_virtual_ranks_match_single_gpu(gpu_available, nranks, structured):
    S, kw = _t64()
    keep, w, rhs = _problem(S, kw)
    x1, st1 = _single(S, keep, w, rhs)
    vd = dist.VirtualDistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, nranks, structured=structured)
    try:
        xd = vd.solve(w, rhs, **TOL)
        std = vd.stats
    finally:
        vd.close()
    assert std['istop'] in (1, 2), std
    assert abs(std['iters'] - st1['iters']) <= max(3, 0.02 * st1['iters']), (std['iters'], st1['iters'])
    assert np.linalg.norm(xd - x1) / np.linalg.norm(x1) <= 1e-8


@pytest.mark.parametrize('structured', [True, False])
def test_virtual_ranks_golden_exact_solution(gpu_available, structured):
    g = golden('sys_sf3d.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    keep, w, rhs = _problem(S, kw)
    vd = dist.VirtualDistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, 2, structured=structured)
    try:
        x = vd.solve(w, rhs, atol=1e-12, btol=1e-12, conlim=1e12, maxit=200000, precond=1)
    finally:
        vd.close()
    xs = g['x']
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) <= 1e-6
    assert np.max(np.abs(x - xs)) <= 1e-4


@pytest.mark.parametrize('structured', [True, False])
def test_virtual_ranks_reweight_and_iterate(gpu_available, structured):
    """Row weights change between solves (the editing loop); fixed-iteration runs work."""
    S, kw = _t64()
    keep, w, rhs = _problem(S, kw)
    vd = dist.VirtualDistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, 2, structured=structured)
    try:
        st = vd.iterate(w, rhs, 40)
        assert st['iters'] == 40
        w2 = w.copy()
        w2[:S['data'].size:7] *= 0.5
        xd = vd.solve(w2, rhs, **TOL)
    finally:
        vd.close()
    x1, _ = _single(S, keep, w2, rhs)
    assert np.linalg.norm(xd - x1) / np.linalg.norm(x1) <= 1e-8


@pytest.mark.parametrize('structured', [True, False])
def test_rccl_one_rank(gpu_available, structured):
    """DistFitSystem over a one-rank RCCL communicator (the N=1 case of bench --gpus N)."""
    import torch.distributed as tdist
    S, kw = _t64()
    keep, w, rhs = _problem(S, kw)
    x1, st1 = _single(S, keep, w, rhs)
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    tdist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    try:
        ds = dist.DistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, 0, 1, device=0, structured=structured)
        try:
            xo = ds.solve(w, rhs, **TOL)
            std = ds.stats
        finally:
            ds.close()
    finally:
        tdist.destroy_process_group()
    x = np.zeros(keep.size)
    ds.scatter_owned(xo, x)
    assert std['istop'] in (1, 2)
    assert np.linalg.norm(x - x1) / np.linalg.norm(x1) <= 1e-8


# ---- CGNR over ranks (lsqr_cg_dist.inc) -------------------------------------------------------
def _single_cg(S, keep, w, rhs, precond):
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    x = fs.solve(w, np.ones(fs.n_data, bool), rhs, atol=1e-12, btol=1e-12, conlim=1e12, precond=precond, method=1)
    st = fs.stats
    fs.close()
    return x, st


@pytest.mark.parametrize('precond,nranks', [(p, n) for p in (3, 1) for n in (2, 3, 4)] + [(4, n) for n in (2, 3, 4, 8)])
def test_virtual_ranks_cgnr_match_single_gpu(gpu_available, nranks, precond):
    """Distributed CGNR (normal-stencil ranks, reverse halo of q, forward halo of z) runs the
    single-GPU recurrence with the same preconditioner (Jacobi from the global column norms;
    block-Jacobi from the node blocks summed over the ranks; multigrid: window level 0 with halos,
    the restriction summed over the ranks, replicated global coarse levels), so the iteration
    counts agree and the solutions match to the solver tolerance."""
    S, kw = _t64()
    keep, w, rhs = _problem(S, kw)
    x1, st1 = _single_cg(S, keep, w, rhs, precond)
    assert st1['method'] == 1
    vd = dist.VirtualDistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, nranks)
    try:
        xd = vd.solve(w, rhs, atol=1e-12, btol=1e-12, conlim=1e12, precond=precond, method=1)
        std = vd.stats
    finally:
        vd.close()
    assert std['method'] == 1 and std['istop'] in (1, 2), std
    slack = 3
    assert abs(std['iters'] - st1['iters']) <= slack, (std['iters'], st1['iters'])
    assert np.linalg.norm(xd - x1) / np.linalg.norm(x1) <= 1e-8


@pytest.mark.parametrize('precond', [3, 1, 4])
def test_virtual_ranks_cgnr_golden_exact_solution(gpu_available, precond):
    g = golden('sys_sf3d.npz')
    kw = golden_kwargs(g)
    S = LS.smooth_fit(data=golden_points(g), return_fit_objects=True, **kw)
    keep, w, rhs = _problem(S, kw)
    vd = dist.VirtualDistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, 2)
    try:
        x = vd.solve(w, rhs, atol=1e-12, btol=1e-12, conlim=1e12, maxit=200000, precond=precond, method=1)
    finally:
        vd.close()
    xs = g['x']
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) <= 1e-6
    assert np.max(np.abs(x - xs)) <= 1e-4


def test_virtual_ranks_cgnr_iterate_matches_solve_prefix(gpu_available):
    """lsq_iterate (fixed iteration count, the bench path) on ranks runs the same iterations as the
    solve: after k iterations the residual estimate equals the solve's after k."""
    S, kw = _t64()
    keep, w, rhs = _problem(S, kw)
    vd = dist.VirtualDistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, 2)
    try:
        st = vd.iterate(w, rhs, 20, precond=3, method=1)
        x = vd.solve(None, None, atol=1e-12, btol=1e-12, conlim=1e12, maxit=20, precond=3, method=1)
        st2 = vd.stats
    finally:
        vd.close()
    assert st['method'] == 1 and st['iters'] == 20 and st2['iters'] == 20
    assert np.isclose(st['r1norm'], st2['r1norm'], rtol=1e-10)
    assert np.all(np.isfinite(x))


def test_virtual_ranks_mg_reweight(gpu_available):
    """Multigrid over ranks across a change of row weights and an edited row mask (the
    editing loop): the per-solve set-up (lumped level-1 data summed over the ranks, λ by power
    steps with halos) follows the new weights; matches the single-GPU multigrid solve."""
    S, kw = _t64()
    keep, w, rhs = _problem(S, kw)
    vd = dist.VirtualDistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, 3)
    w2 = w.copy()
    w2[:S['data'].size:5] = 0.0        # edited data rows carry weight 0
    w2[1:S['data'].size:7] *= 2.0
    try:
        vd.solve(w, rhs, atol=1e-12, btol=1e-12, conlim=1e12, precond=4, method=1)
        xd = vd.solve(w2, rhs, atol=1e-12, btol=1e-12, conlim=1e12, precond=4, method=1)
        std = vd.stats
    finally:
        vd.close()
    x1, st1 = _single_cg(S, keep, w2, rhs, 4)
    assert abs(std['iters'] - st1['iters']) <= 3, (std['iters'], st1['iters'])
    assert np.linalg.norm(xd - x1) / np.linalg.norm(x1) <= 1e-8
