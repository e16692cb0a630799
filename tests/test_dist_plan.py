"""Host side of the multi-GPU path (lssurf_amd.dist): y-slab partition, per-rank row
descriptors, column ownership, ghost layout and exchange plans.  CPU only; the world_size-2
case runs the plan exchange over torch.distributed (gloo) exactly as DistFitSystem does."""
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sp

import lssurf_amd as LS
from lssurf_amd import dist, synthetic
from lssurf_amd.constraint_functions import reference_epoch_keep_cols


def _system(name='t64'):
    D, kw = synthetic.points(name)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    return S, keep


def _host_csr(S, keep):
    A = sp.vstack([S['G_data'].toCSR(), S['Gc'].toCSR()]).tocsr()[:, keep].tocsr()
    A.eliminate_zeros()
    return A


def _flags(A, rows):
    f = np.zeros(A.shape[1], np.uint8)
    f[np.unique(A[rows].indices)] = 1
    return f


@pytest.mark.parametrize('nranks', [1, 2, 3, 5])
def test_rows_partitioned_exactly_once(nranks):
    S, keep = _system()
    part = dist.SlabPartition(S['grids']['dz'], nranks)
    m = S['G_data'].N_eq + S['Gc'].N_eq
    probs = [dist.rank_problem(S['G_data'], S['Gc'], part, r) for r in range(nranks)]
    allrows = np.concatenate([p['rows'] for p in probs])
    np.testing.assert_array_equal(np.sort(allrows), np.arange(m))
    for p in probs:
        assert p['m'] == p['rows'].size
        assert p['npts'] + sum(s.n_eq for s in p['stencils']) == p['m']
        assert np.all(np.diff(p['rows'][:p['npts']]) > 0)


@pytest.mark.parametrize('nranks', [2, 4])
def test_ghosts_only_from_neighbouring_slabs(nranks):
    S, keep = _system()
    A = _host_csr(S, keep)
    part = dist.SlabPartition(S['grids']['dz'], nranks)
    probs = [dist.rank_problem(S['G_data'], S['Gc'], part, r) for r in range(nranks)]
    owner = dist.column_owner(keep, probs[0]['grid_objs'], part)
    assert np.bincount(owner, minlength=nranks).min() > 0
    lays = [dist.local_layout(_flags(A, p['rows']), owner, r) for r, p in enumerate(probs)]
    for r, lay in enumerate(lays):
        col_local, n_local, n_own, ghosts, owned = lay
        assert set(ghosts) <= {r - 1, r + 1}
        assert n_own == owned.size and n_local == n_own + sum(g.size for g in ghosts.values())
        np.testing.assert_array_equal(col_local[owned], np.arange(n_own))
    # owned sets tile the columns; every column is referenced by some rank's rows
    np.testing.assert_array_equal(np.sort(np.concatenate([l[4] for l in lays])), np.arange(keep.size))


def test_exchange_plans_are_mirrored():
    S, keep = _system()
    A = _host_csr(S, keep)
    nr = 3
    part = dist.SlabPartition(S['grids']['dz'], nr)
    probs = [dist.rank_problem(S['G_data'], S['Gc'], part, r) for r in range(nr)]
    owner = dist.column_owner(keep, probs[0]['grid_objs'], part)
    lays = [dist.local_layout(_flags(A, p['rows']), owner, r) for r, p in enumerate(probs)]
    ghosts_of = [l[3] for l in lays]
    plans = [dist.exchange_plan(r, lays[r][0], ghosts_of) for r in range(nr)]
    _check_mirrored(lays, plans)


def _check_mirrored(lays, plans):
    nr = len(lays)
    for r in range(nr):
        peers, send_cnt, send_idx, recv_cnt = plans[r]
        off = np.r_[0, np.cumsum(send_cnt)]
        for k, p in enumerate(peers):
            pk = list(plans[p][0]).index(r)
            assert send_cnt[k] == plans[p][3][pk]          # what r sends is what p receives
            owned_r = lays[r][4]
            sent_global = owned_r[send_idx[off[k]:off[k + 1]]]
            np.testing.assert_array_equal(sent_global, lays[p][3][r])   # in p's ghost-slot order


def _worker(rank, world, port, outq):
    import torch.distributed as tdist
    tdist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    try:
        S, keep = _system()
        A = _host_csr(S, keep)
        part = dist.SlabPartition(S['grids']['dz'], world)
        prob = dist.rank_problem(S['G_data'], S['Gc'], part, rank)
        owner = dist.column_owner(keep, prob['grid_objs'], part)
        lay = dist.local_layout(_flags(A, prob['rows']), owner, rank)
        gathered = [None] * world
        tdist.all_gather_object(gathered, lay[3])
        plan = dist.exchange_plan(rank, lay[0], gathered)
        allp = [None] * world
        tdist.all_gather_object(allp, (lay, plan))
        if rank == 0:
            _check_mirrored([a[0] for a in allp], [a[1] for a in allp])
        outq.put((rank, 'ok'))
    except Exception as e:   # report to the parent
        outq.put((rank, repr(e)))
    finally:
        tdist.destroy_process_group()


def test_gloo_world2_plan_exchange():
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: 'ok', 1: 'ok'}, res


@pytest.mark.parametrize('nranks', [2, 3, 4])
def test_windows_partition_rows_and_columns(nranks):
    """Structured-operator ranks: every row in exactly one window, owned columns tile the
    compact space, halo lists mirror each other (same global columns, same order)."""
    S, keep = _system()
    part = dist.SlabPartition(S['grids']['dz'], nranks)
    m = S['G_data'].N_eq + S['Gc'].N_eq
    probs = [dist.window_problem(S['G_data'], S['Gc'], part, r, keep) for r in range(nranks)]
    np.testing.assert_array_equal(np.sort(np.concatenate([p['rows'] for p in probs])), np.arange(m))
    x = np.zeros(keep.size)
    for p in probs:
        dist.window_owned_solution(p, np.ones(p['keep'].size), x)
    assert np.all(x == 1.0)
    assert sum(int(np.sum([b - a for a, b in p['own_ranges']])) for p in probs) == S['Gc'].col_N
    halos = [dist.window_halo(p['grid_objs'], part, r, p['halo']) for r, p in enumerate(probs)]
    for r, (peers, sc, si, rc, ri) in enumerate(halos):
        so, ro = np.r_[0, np.cumsum(sc)], np.r_[0, np.cumsum(rc)]
        for k, q in enumerate(peers):
            pq = halos[q]
            kk = list(pq[0]).index(r)
            qso = np.r_[0, np.cumsum(pq[1])]
            mine_sent = probs[r]['l2g'][si[so[k]:so[k + 1]]]
            theirs_recv = probs[q]['l2g'][pq[4][np.r_[0, np.cumsum(pq[3])][kk]:np.r_[0, np.cumsum(pq[3])][kk + 1]]]
            np.testing.assert_array_equal(mine_sent, theirs_recv)
            assert np.all(np.diff(mine_sent) > 0)


@pytest.mark.parametrize('nranks', [2, 3])
def test_window_node_blocks_cover_window_in_global_order(nranks):
    """Block-Jacobi blocks of a rank (dist.window_node_blocks): one block per window node
    (owned and ghost), in local compact ids whose global columns are exactly the single-GPU node
    block of that node — same columns in the same order on every rank holding the node, which
    is what lets group_block_factor sum the partial (AᵀA)_bb column by column."""
    from lssurf_amd.constraint_functions import node_column_blocks
    S, keep = _system()
    part = dist.SlabPartition(S['grids']['dz'], nranks)
    gptr, gcols = node_column_blocks(S['grids'], keep)
    gblocks = {tuple(keep[gcols[gptr[b]:gptr[b + 1]]]) for b in range(gptr.size - 1)}
    seen = {}
    for r in range(nranks):
        prob = dist.window_problem(S['G_data'], S['Gc'], part, r, keep)
        bptr, bcols = dist.window_node_blocks(prob, keep)
        assert bptr[0] == 0 and np.all(np.diff(bptr) > 0) and bcols.max() < prob['keep'].size
        glob = prob['l2g'][prob['keep'][bcols]]                # local compact -> global full ids
        for b in range(bptr.size - 1):
            blk = tuple(glob[bptr[b]:bptr[b + 1]])
            assert blk in gblocks
            seen.setdefault(blk, set()).add(r)
        assert np.unique(bcols).size == bcols.size            # a column in at most one block
    assert set(seen) == gblocks                               # every node block lives on some rank
    assert any(len(v) > 1 for v in seen.values())             # halo nodes are shared


@pytest.mark.parametrize('name,nranks,base', [('c4y4', 4, 'c4'), ('c4y8', 8, 'c4'), ('c5y8', 8, 'c5')])
def test_slab_configs_are_one_rank_window_of_c4(name, nranks, base):
    """synthetic 'c4y4' / 'c4y8' / 'c5y8' (the per-rank compute floor of bench --gpus 4 / 8 on C4
    and C5): the node-row count of one interior rank's window (owned rows + halo
    rows), the full config's row width, epochs and spacing, and 1/N of its points."""
    from lssurf_amd import synthetic
    n, nt, npts = synthetic.CONFIGS[base]
    kw, pts = synthetic.config_kwargs(name)
    ck, cpts = synthetic.config_kwargs(base)
    assert pts * nranks == cpts and kw['spacing'] == ck['spacing'] and kw['W']['x'] == ck['W']['x']
    ny = int(round(kw['W']['y'] / kw['spacing']['dz'])) + 1
    halo = 1   # one ghost node row per side (the stencils and the interpolation reach one row)
    assert ny == n // nranks + 2 * halo
    D, _ = synthetic.points(name)
    assert D.size == pts and np.all(np.abs(D.y) <= kw['W']['y'] / 2) and np.all(np.abs(D.x) <= kw['W']['x'] / 2)


def test_window_problem_slices_field_values():
    """Field-valued parts (the anisotropic directional operator) over y-slab windows: every
    rank keeps the rows of its owned centres and exactly their field values; the ranks' rows
    tile the global rows once."""
    from lssurf_amd import assemble, dist, synthetic
    S, kw = synthetic.aniso_system('ta64')
    d = assemble.describe(S['G_data'], S['Gc'], with_fields=True)
    stencils, npts, fields = d[3], d[4], d[5]
    (k, off, val, fsel, F), = fields
    s = stencils[k]
    part = dist.SlabPartition(S['grids']['dz'], 3)
    seen = []
    for r in range(3):
        prob = dist.window_problem(S['G_data'], S['Gc'], part, r, S['keep'])
        seen.append(prob['rows'])
        (kl, offl, vall, fsell, Fl), = prob['fields']
        t = prob['stencils'][kl]
        rows = prob['rows'][t.row0:t.row0 + t.n_eq] - int(s.row0)     # the part's global row indices
        assert np.array_equal(offl, off) and np.array_equal(Fl, F[:, rows])
        assert prob['halo'] >= 1
    allrows = np.sort(np.concatenate(seen))
    assert np.array_equal(allrows, np.arange(S['w'].size))


def test_synthetic_seed_ids_frozen():
    """Every synthetic config has its own frozen seed offset (SEED_ID), independent of the order of
    CONFIGS: a config added anywhere must not move the points of the others (round 3's position-
    derived offsets did: C5a's cloud changed under the benchmark)."""
    from lssurf_amd import synthetic
    assert set(synthetic.SEED_ID) == set(synthetic.CONFIGS)
    assert len(set(synthetic.SEED_ID.values())) == len(synthetic.SEED_ID)
    assert synthetic.SEED_ID['c4'] == 2 and synthetic.SEED_ID['c5a'] == 11


def test_node_column_blocks_uniform_fast_path():
    """node_column_blocks' fast path (the same kept columns at every node: views of the compact-
    position map) returns exactly what the general path does — shared lattice, 15 epochs, z0 on a
    2× refinement (dz-only blocks)."""
    from lssurf_amd import constraint_functions as cf
    import lssurf_amd as LS
    for name in ('t64', 't15', 't64z'):
        D, kw = synthetic.points(name)
        S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
        keep = np.asarray(cf.reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch']))
        fast = cf._node_column_blocks_uniform(S['grids']['z0'], S['grids']['dz'], keep, 16)
        assert fast is not None, name
        saved = cf._node_column_blocks_uniform
        try:
            cf._node_column_blocks_uniform = lambda *a: None
            ref = cf.node_column_blocks(S['grids'], keep)
        finally:
            cf._node_column_blocks_uniform = saved
        assert np.array_equal(fast[0], ref[0]) and np.array_equal(fast[1], ref[1]), name
        assert fast[1].dtype == np.int32 and fast[0].dtype == np.int64


def test_node_column_blocks_affine_matches_explicit():
    """The affine form of the node blocks (lsq_set_column_blocks_affine) expands to exactly
    node_column_blocks' (block_ptr, cols); systems whose blocks leave singleton columns (z0 on a
    2× refinement) or whose kept set is not the same at every node get None (explicit path)."""
    from lssurf_amd import constraint_functions as cf
    import lssurf_amd as LS
    for name in ('t64', 't15', 't64z'):
        D, kw = synthetic.points(name)
        S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
        keep = np.asarray(cf.reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch']))
        ref = cf.node_column_blocks(S['grids'], keep)
        aff = cf.node_column_blocks_affine(S['grids'], keep)
        if name == 't64z':
            assert aff is None
            continue
        nb, base, stride, fbase, fstride = aff
        b = np.arange(nb)[:, None]
        cols = base[None, :] + b * stride[None, :]
        np.testing.assert_array_equal(ref[0], np.arange(nb + 1) * base.size)
        np.testing.assert_array_equal(ref[1], cols.ravel())
        np.testing.assert_array_equal(keep[cols], fbase[None, :] + b * fstride[None, :])
        hole = np.delete(keep, keep.size // 2)          # one node short of a column
        assert cf.node_column_blocks_affine(S['grids'], hole) is None
