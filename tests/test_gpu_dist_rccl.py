"""Two RCCL ranks in two processes on the one GPU of the test box.

RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"), so each rank
declares its own host id (NCCL_HOSTID) and the ranks talk over the socket transport on the
loopback interface.  The kernels, halos (ncclSend/ncclRecv groups) and all-reduces are the ones
an 8-GPU node runs over xGMI; only the wire differs.  The distributed solution must match the
single-GPU solve to the solver tolerance (≤1e-8 relative at atol = btol = 1e-12)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = dict(atol=1e-12, btol=1e-12, conlim=1e12, precond=1)


def _problem():
    import lssurf_amd as LS
    from lssurf_amd import synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    D, kw = synthetic.points('t64')
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    E_all = 1 / (1. / np.concatenate((S['Ed'], S['Ec'])))
    w = 1. / np.sqrt(E_all ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    return S, keep, w, rhs


def _rank(rank, world, port, structured, outq, opts=TOL):
    os.environ['NCCL_HOSTID'] = f'lsq-test-host-{rank}'
    os.environ.setdefault('NCCL_SOCKET_IFNAME', 'lo')
    os.environ.setdefault('NCCL_IB_DISABLE', '1')
    import torch.distributed as tdist
    from lssurf_amd import dist
    tdist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    try:
        S, keep, w, rhs = _problem()
        ds = dist.DistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, rank, world, device=0,
                                structured=structured)
        try:
            xl = ds.solve(w, rhs, **opts)
            st = ds.stats
        finally:
            ds.close()
        x = np.zeros(keep.size)
        ds.scatter_owned(xl, x)
        outq.put((rank, x, st['iters'], st['istop']))
    except Exception as e:   # report to the parent
        outq.put((rank, repr(e), -1, -1))
    finally:
        tdist.destroy_process_group()


CG_TOL = dict(atol=1e-12, btol=1e-12, conlim=1e12, precond=3, method=1)


MG_TOL = dict(CG_TOL, precond=4)


@pytest.mark.parametrize('structured,opts', [(True, TOL), (False, TOL), (True, CG_TOL), (True, MG_TOL)],
                         ids=['lsqr-structured', 'lsqr-assembled', 'cgnr-blockjacobi', 'cgnr-multigrid'])
def test_two_rccl_ranks_match_single_gpu(gpu_available, structured, opts):
    """cgnr-blockjacobi: CGNR + block-Jacobi over RCCL (halos of q and z, two all-reduces per
    iteration, node blocks summed over the ranks before factoring); cgnr-multigrid: the V-cycle
    over RCCL (level-0 halos, the restricted residual all-reduced once per cycle)."""
    import torch.multiprocessing as mp
    from lssurf_amd.smooth_fit import FitSystem
    S, keep, w, rhs = _problem()
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    x1 = fs.solve(w, np.ones(fs.n_data, bool), rhs, **opts)
    it1 = fs.stats['iters']
    fs.close()
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, structured, q, opts)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=400) for _ in procs]
    for p in procs:
        p.join(60)
    for r, x, it, istop in res:
        assert not isinstance(x, str), x
    x = sum(r[1] for r in res)
    assert all(r[3] in (1, 2) for r in res)
    assert abs(res[0][2] - it1) <= max(3, 0.02 * it1)
    assert np.linalg.norm(x - x1) / np.linalg.norm(x1) <= 1e-8
