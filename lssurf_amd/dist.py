"""Multi-GPU smooth_fit solve: y-slab partition of one least-squares system over ranks.

SURVEY.md §8(e): every rank owns the unknowns (z0 and dz columns) of a band of node rows and
the equations anchored there (stencil rows by their centre node, data rows by the point's y);
stencils and the bilinear/trilinear interpolation reach one node row across a slab boundary,
so a rank's rows touch one "ghost" node row per side.  The device solve then needs, per LSQR
iteration, one forward halo (ghost ṽ before A·v), one reverse halo (ghost partial sums after
Aᵀu) and two all-reduces of 1–2 doubles — liblsqsurf does those with RCCL over xGMI
(``DistFitSystem``, one process per GPU) or, for testing on one GPU, between in-process
virtual ranks (``VirtualDistFitSystem``).  Nothing here copies matrices between ranks: each
rank's device generates its own rows from the shared grid/stencil description.
"""
import ctypes

import numpy as np

from . import assemble
from ._native import LsqStats, NativeError, as_c, default_opts, load, ptr
from .solver import LSQSolver


class SlabPartition:
    """Node-row bands of the dz grid (the bulk of the unknowns); every other grid's rows, the
    stencil centres and the data points follow by their y coordinate."""

    def __init__(self, grid, nranks):
        ny = int(grid.shape[0])
        if nranks > ny:
            raise ValueError(f'{nranks} ranks for {ny} node rows')
        cuts = [int(round(k * ny / nranks)) for k in range(1, nranks)]
        self.bounds = np.array([grid.ctrs[0][0] + (c - 0.5) * grid.delta[0] for c in cuts])
        self.nranks = nranks

    def owner(self, y):
        return np.searchsorted(self.bounds, y, side='right')

    def rows_of(self, grid, rank):
        """[a, b): the node rows of `grid` owned by `rank` (contiguous)."""
        own = np.flatnonzero(self.owner(grid.ctrs[0]) == rank)
        return (int(own[0]), int(own[-1]) + 1) if own.size else (0, 0)


def rank_problem(G_data, Gc, partition, rank):
    """Descriptors of the rows `rank` owns + their global row ids (None: not structured)."""
    desc = assemble.describe(G_data, Gc)
    if desc is None:
        raise NotImplementedError('distributed solve on assembled ranks needs a constant-coefficient stencil system '
                                  '(field-valued parts: structured ranks)')
    grid_descs, interp, (py, px, pt), stencils, npts = desc
    grid_objs = {}
    for p in list(G_data.parts) + list(Gc.parts):
        grid_objs[id(p['grid'])] = p['grid']
    # the descriptor order of describe() is first-seen order over G_data then Gc parts
    order, seen = [], set()
    for p in list(G_data.parts) + list(Gc.parts):
        if id(p['grid']) not in seen:
            seen.add(id(p['grid']))
            order.append(p['grid'])
    pts_own = np.flatnonzero(partition.owner(py) == rank)
    rows = [pts_own]
    local = []
    row0 = pts_own.size
    for s, part in zip(stencils, Gc.parts):
        g = order[s.grid]
        a, b = partition.rows_of(g, rank)
        lo_y, hi_y = max(int(s.lo[0]), a), min(int(s.hi[0]), b)
        if lo_y >= hi_y:
            continue
        nd = int(g.N_dims)
        inner = int(np.prod([int(s.hi[d]) - int(s.lo[d]) for d in range(1, nd)]))
        t = type(s).from_buffer_copy(s)
        t.lo[0], t.hi[0] = lo_y, hi_y
        t.n_eq = (hi_y - lo_y) * inner
        t.row0 = row0
        first = npts + int(part['row0']) + (lo_y - int(s.lo[0])) * inner
        rows.append(first + np.arange(t.n_eq))
        row0 += t.n_eq
        local.append(t)
    coords = (py[pts_own].copy(), px[pts_own].copy(), None if pt is None else pt[pts_own].copy())
    return dict(grids=grid_descs, grid_objs=order, interp=interp, coords=coords, stencils=local,
                npts=int(pts_own.size), rows=np.concatenate(rows), m=int(row0))


def _describe_order(G_data, Gc):
    desc = assemble.describe(G_data, Gc, with_fields=True)
    if desc is None:
        raise NotImplementedError('distributed solve needs a structured (stencil + interp) system')
    order, seen = [], set()
    for p in list(G_data.parts) + list(Gc.parts):
        if id(p['grid']) not in seen:
            seen.add(id(p['grid']))
            order.append(p['grid'])
    return desc, order


def window_meta(grid_objs, partition, rank, halo):
    """Per grid: (wa, wb, a, b) = window rows [wa, wb) = owned rows [a, b) ± halo rows, and the
    local column offset of the grid's window (grids in global column order)."""
    meta, col0 = [], 0
    for g in grid_objs:
        a, b = partition.rows_of(g, rank)
        if a >= b:
            raise ValueError(f'rank {rank} owns no node rows of a grid: too many ranks for the grid')
        ny = int(g.shape[0])
        wa, wb = max(0, a - halo), min(ny, b + halo)
        stride = int(g.stride[0])
        meta.append(dict(wa=wa, wb=wb, a=a, b=b, stride=stride, col0=col0, gcol0=int(g.col_0)))
        col0 += (wb - wa) * stride
    return meta, col0


def window_problem(G_data, Gc, partition, rank, keep_cols):
    """The rank's window of the structured system: sub-grids of its owned node rows ± halo rows
    (own column numbering), the stencil parts clipped to its owned centre rows, its points, and
    the maps to the global system.  Every rank computes every window (no communication)."""
    from ._native import GridDesc
    (grid_descs, interp, (py, px, pt), stencils, npts, fields), order = _describe_order(G_data, Gc)
    fields = {f[0]: f for f in fields}            # field-valued parts by stencil index
    halo = max([1] + [abs(int(s.off[t][0])) for k, s in enumerate(stencils) if k not in fields for t in range(s.ntpl)]
               + [int(np.abs(f[1][:, 0]).max()) for f in fields.values()])
    meta, nloc = window_meta(order, partition, rank, halo)
    grids = []
    for gd, gm in zip(grid_descs, meta):
        d = GridDesc.from_buffer_copy(gd)
        d.shape[0] = gm['wb'] - gm['wa']
        d.b0[0] = gd.b0[0] + gm['wa'] * gd.delta[0]
        d.col0 = gm['col0']
        grids.append(d)
    pts_own = np.flatnonzero(partition.owner(py) == rank)
    rows = [pts_own]
    local, local_fields, part_rows = [], [], []
    row0 = pts_own.size
    for k, s in enumerate(stencils):
        gm = meta[s.grid]
        lo_y, hi_y = max(int(s.lo[0]), gm['a']), min(int(s.hi[0]), gm['b'])
        if lo_y >= hi_y:
            continue
        nd = int(order[s.grid].N_dims)
        inner = int(np.prod([int(s.hi[d]) - int(s.lo[d]) for d in range(1, nd)]))
        t = type(s).from_buffer_copy(s)
        t.lo[0], t.hi[0] = lo_y - gm['wa'], hi_y - gm['wa']
        t.n_eq = (hi_y - lo_y) * inner
        t.row0 = row0
        k0 = (lo_y - int(s.lo[0])) * inner            # first of the part's rows kept (centre order)
        first = int(s.row0) + k0
        rows.append(first + np.arange(t.n_eq))
        part_rows.append((row0, first, t.n_eq))       # local rows [row0, +n) = global rows [first, +n)
        if k in fields:                               # the kept rows' field values
            _, off, val, fsel, F = fields[k]
            local_fields.append((len(local), off, val, fsel, np.ascontiguousarray(F[:, k0:k0 + t.n_eq])))
        row0 += t.n_eq
        local.append(t)
    coords = (py[pts_own].copy(), px[pts_own].copy(), None if pt is None else pt[pts_own].copy())
    l2g = np.concatenate([gm['gcol0'] + gm['wa'] * gm['stride'] + np.arange((gm['wb'] - gm['wa']) * gm['stride'])
                          for gm in meta])
    keep_cols = np.asarray(keep_cols)
    pos = np.minimum(np.searchsorted(keep_cols, l2g), keep_cols.size - 1)
    keep_local = np.flatnonzero(keep_cols[pos] == l2g)
    own_ranges = [(gm['col0'] + (gm['a'] - gm['wa']) * gm['stride'], gm['col0'] + (gm['b'] - gm['wa']) * gm['stride'])
                  for gm in meta]
    # the global description (multigrid over ranks: replicated coarse levels, lsq_dist_set_global)
    gst, local_of, nl = [], [], 0
    for k, s in enumerate(stencils):
        t = type(s).from_buffer_copy(s)
        if k in fields:
            t.ntpl = 0                                # field-valued: its coarse rows come from the ranks
        gst.append(t)
        gm = meta[s.grid]
        if max(int(s.lo[0]), gm['a']) < min(int(s.hi[0]), gm['b']):
            local_of.append(nl)
            nl += 1
        else:
            local_of.append(-1)
    lat = {(gm['wa'], gm['a'], gm['b'], int(g.shape[0])) for gm, g in zip(meta, order)}
    glob = None
    if len(lat) == 1:                                 # one (y, x) lattice shared by the grids
        wa, a, b, ny = lat.pop()
        glob = dict(grids=list(grid_descs), stencils=gst, local_of=np.array(local_of, np.int32), wa=wa, oa=a, ob=b,
                    rows=ny, n_full=int(max(int(g.col_0) + int(g.N_nodes) for g in order)))
    return dict(grids=grids, grid_objs=order, interp=interp, coords=coords, stencils=local, fields=local_fields,
                npts=int(pts_own.size), rows=np.concatenate(rows), part_rows=part_rows, m=int(row0), n_full=int(nloc),
                keep=keep_local, l2g=l2g,
                keep_global=pos[keep_local], own_ranges=own_ranges, meta=meta, halo=halo, glob=glob)


def window_halo(grid_objs, partition, rank, halo):
    """Halo lists of `rank` (local full ids, ascending global order): per peer, the owned
    columns the peer holds as ghosts (send) and the ghost columns the peer owns (recv)."""
    nr = partition.nranks
    metas = [window_meta(grid_objs, partition, r, halo)[0] for r in range(nr)]
    mine = metas[rank]
    peers, send, recv = [], [], []
    for p in range(nr):
        if p == rank:
            continue
        s_ids, r_ids = [], []
        for gm, gp in zip(mine, metas[p]):
            lo, hi = max(gm['a'], gp['wa']), min(gm['b'], gp['wb'])        # my owned rows in p's window
            if lo < hi:
                s_ids.append(gm['col0'] + (lo - gm['wa']) * gm['stride'] + np.arange((hi - lo) * gm['stride']))
            lo, hi = max(gm['wa'], gp['a']), min(gm['wb'], gp['b'])        # p's owned rows in my window
            if lo < hi:
                r_ids.append(gm['col0'] + (lo - gm['wa']) * gm['stride'] + np.arange((hi - lo) * gm['stride']))
        if s_ids or r_ids:
            peers.append(p)
            send.append(np.concatenate(s_ids) if s_ids else np.zeros(0, np.int64))
            recv.append(np.concatenate(r_ids) if r_ids else np.zeros(0, np.int64))
    cat = lambda xs: np.concatenate(xs).astype(np.int32) if xs else np.zeros(0, np.int32)
    return (np.array(peers, np.int32), np.array([x.size for x in send], np.int64), cat(send),
            np.array([x.size for x in recv], np.int64), cat(recv))


def _form_window(L, h, prob):
    from ._native import GridDesc, StencilDesc
    s = _HandleView(L, h)
    keep = as_c(prob['keep'], np.int64)
    s.check(L.lsq_set_col_map(h, prob['n_full'], ptr(keep), keep.size), 'lsq_set_col_map')
    ga = (GridDesc * len(prob['grids']))(*prob['grids'])
    sa = (StencilDesc * max(len(prob['stencils']), 1))(*prob['stencils'])
    ig = as_c(np.asarray(prob['interp'], np.int32), np.int32)
    py, px, pt = prob['coords']
    for k, off, val, fsel, F in prob.get('fields', ()):
        off, val, fsel = as_c(off, np.int32).reshape(-1, 3), as_c(val, np.float64), as_c(fsel, np.int32)
        F = as_c(F, np.float64)
        s.check(L.lsq_set_stencil_fields(h, int(k), off.shape[0], ptr(off), ptr(val), F.shape[0], ptr(fsel), F.shape[1],
                                         ptr(F)), 'lsq_set_stencil_fields')
    s.check(L.lsq_set_matrix_stencil(h, prob['m'], prob['n_full'], len(prob['grids']),
                                     ctypes.cast(ga, ctypes.c_void_p), len(prob['interp']), ptr(ig), prob['npts'],
                                     ptr(py), ptr(px), ptr(pt), len(prob['stencils']), ctypes.cast(sa, ctypes.c_void_p),
                                     None), 'lsq_set_matrix_stencil')


def _install_halo(L, h, prob, halo):
    peers, send_cnt, send_idx, recv_cnt, recv_idx = halo
    rng = as_c(np.asarray(prob['own_ranges'], np.int64).ravel(), np.int64)
    _HandleView(L, h).check(
        L.lsq_dist_set_halo(h, len(prob['own_ranges']), ptr(rng), peers.size, ptr(peers), ptr(send_cnt),
                            ptr(send_idx), ptr(recv_cnt), ptr(recv_idx)), 'lsq_dist_set_halo')


def _install_global(L, h, prob):
    """The global grids and parts + the rank's place in them (multigrid, precond 4).  A system the
    device cannot describe globally keeps precond 1/3; precond 4 then reports why."""
    from ._native import GridDesc, StencilDesc
    g = prob.get('glob')
    if g is None:
        return False
    ga = (GridDesc * len(g['grids']))(*g['grids'])
    sa = (StencilDesc * max(len(g['stencils']), 1))(*g['stencils'])
    lo = as_c(g['local_of'], np.int32)
    rc = L.lsq_dist_set_global(h, g['n_full'], len(g['grids']), ctypes.cast(ga, ctypes.c_void_p), len(g['stencils']),
                               ctypes.cast(sa, ctypes.c_void_p), ptr(lo), g['wa'], g['oa'], g['ob'], g['rows'])
    return rc == 0


def window_node_blocks(prob, keep_cols):
    """Block-Jacobi blocks (precond 3) of a rank: the node blocks of constraint_functions.
    node_column_blocks for every node of the rank's window (owned and ghost), in the rank's local
    compact column ids (block_ptr, cols), or None when the grids have no node-block structure.
    The ghost blocks carry the rank's partial (AᵀA)_bb to their owners (group_block_factor); the
    update kernels skip ghost columns."""
    from .constraint_functions import node_column_blocks
    grids = {}
    for g in prob['grid_objs']:
        grids['dz' if g.N_dims == 3 else 'z0'] = g
    blocks = node_column_blocks(grids, keep_cols)
    if blocks is None:
        return None
    bptr, bcols = blocks
    keep_cols = np.asarray(keep_cols)
    l2g = prob['l2g']
    gfull = keep_cols[bcols]
    lf = np.minimum(np.searchsorted(l2g, gfull), l2g.size - 1)
    ok = l2g[lf] == gfull
    keep_local = np.asarray(prob['keep'])
    lc = np.minimum(np.searchsorted(keep_local, lf), keep_local.size - 1)
    ok &= keep_local[lc] == lf
    lens = np.diff(bptr)
    blk_ok = np.add.reduceat(ok.astype(np.int64), bptr[:-1]) == lens   # every column in the window and kept
    sel = np.repeat(blk_ok, lens)
    return np.r_[0, np.cumsum(lens[blk_ok])].astype(np.int64), lc[sel].astype(np.int32)


def _install_blocks(L, h, prob, keep_cols):
    blocks = window_node_blocks(prob, keep_cols)
    if blocks is None:
        return False
    bptr, bcols = blocks
    _HandleView(L, h).check(L.lsq_set_column_blocks(h, bptr.size - 1, ptr(bptr), ptr(bcols)), 'lsq_set_column_blocks')
    return True


def window_owned_solution(prob, x_local, x_out):
    """Scatter the owned columns of a rank's local compact solution into the global compact x."""
    full = prob['keep']
    own = np.zeros(prob['n_full'], bool)
    for a, b in prob['own_ranges']:
        own[a:b] = True
    sel = own[full]
    x_out[prob['keep_global'][sel]] = x_local[sel]


def column_owner(keep_cols, grid_objs, partition):
    """Owner rank of every compact column (global full column -> its grid node row -> y)."""
    full = np.asarray(keep_cols)
    owner = np.empty(full.size, dtype=np.int32)
    done = np.zeros(full.size, dtype=bool)
    for g in grid_objs:
        sel = (full >= g.col_0) & (full < g.col_0 + g.N_nodes)
        iy = (full[sel] - g.col_0) // int(g.stride[0])
        owner[sel] = partition.owner(g.ctrs[0][iy])
        done |= sel
    if not done.all():
        raise ValueError('columns outside every grid')
    return owner


def local_layout(flags, owner, rank):
    """col_local (compact -> local id), n_local, n_own, ghosts {peer: sorted compact ids}."""
    owned = np.flatnonzero(owner == rank)
    ghost = np.flatnonzero(flags.astype(bool) & (owner != rank))
    ghosts = {}
    pieces = [owned]
    for p in np.unique(owner[ghost]):
        ids = ghost[owner[ghost] == p]
        ghosts[int(p)] = ids
        pieces.append(ids)
    order = np.concatenate(pieces)
    col_local = np.full(owner.size, -1, dtype=np.int32)
    col_local[order] = np.arange(order.size, dtype=np.int32)
    return col_local, int(order.size), int(owned.size), ghosts, owned


def exchange_plan(rank, col_local, ghosts_of):
    """Per-peer send lists (owned local ids, in the peer's ghost order) and receive counts."""
    mine = ghosts_of[rank]
    peers = sorted(set(mine) | {p for p, g in enumerate(ghosts_of) if rank in g})
    send_cnt, send_idx, recv_cnt = [], [], []
    for p in peers:
        want = ghosts_of[p].get(rank, np.zeros(0, dtype=np.int64))
        send_cnt.append(want.size)
        send_idx.append(col_local[want])
        recv_cnt.append(mine.get(p, np.zeros(0)).size)
    send_idx = np.concatenate(send_idx).astype(np.int32) if send_idx else np.zeros(0, np.int32)
    return (np.array(peers, dtype=np.int32), np.array(send_cnt, dtype=np.int64), send_idx,
            np.array(recv_cnt, dtype=np.int64))


def _form_rank(L, h, prob, keep_cols, n_full):
    from ._native import GridDesc, StencilDesc
    s = _HandleView(L, h)
    keep = as_c(keep_cols, np.int64)
    s.check(L.lsq_set_col_map(h, int(n_full), ptr(keep), keep.size), 'lsq_set_col_map')
    ga = (GridDesc * len(prob['grids']))(*prob['grids'])
    sa = (StencilDesc * max(len(prob['stencils']), 1))(*prob['stencils'])
    ig = as_c(np.asarray(prob['interp'], np.int32), np.int32)
    py, px, pt = prob['coords']
    s.check(L.lsq_set_matrix_stencil(h, prob['m'], int(n_full), len(prob['grids']), ctypes.cast(ga, ctypes.c_void_p),
                                     len(prob['interp']), ptr(ig), prob['npts'], ptr(py), ptr(px), ptr(pt),
                                     len(prob['stencils']), ctypes.cast(sa, ctypes.c_void_p), None),
            'lsq_set_matrix_stencil')
    flags = np.zeros(keep.size, np.uint8)
    s.check(L.lsq_dist_referenced_cols(h, ptr(flags)), 'lsq_dist_referenced_cols')
    return flags


def _install_layout(L, h, lay, plan):
    col_local, n_local, n_own = lay[:3]
    peers, send_cnt, send_idx, recv_cnt = plan
    _HandleView(L, h).check(
        L.lsq_dist_set_layout(h, ptr(col_local), n_local, n_own, peers.size, ptr(peers), ptr(send_cnt), ptr(send_idx),
                              ptr(recv_cnt)), 'lsq_dist_set_layout')


class _HandleView:
    def __init__(self, L, h):
        self.L, self.h = L, h

    def check(self, rc, what):
        if rc < 0:
            raise NativeError(f'{what}: {self.L.lsq_last_error(self.h).decode()}')
        return rc


def _quiet_stdout(fn):
    """RCCL prints a version banner on stdout at communicator creation; send it to stderr so a
    rank's stdout stays machine-readable (bench.py prints exactly one JSON line)."""
    import os
    import sys
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        return fn()
    finally:
        os.dup2(saved, 1)
        os.close(saved)


class _Base:
    def _setup_common(self, G_data, Gc, keep_cols, n_full, nranks):
        dz = [g for g in (p['grid'] for p in Gc.parts) if g.N_dims == 3]
        base_grid = dz[0] if dz else Gc.parts[0]['grid']
        self.partition = SlabPartition(base_grid, nranks)
        self.keep_cols = np.asarray(keep_cols)
        self.n_full = int(n_full)
        self.n_data = int(G_data.N_eq)


class DistFitSystem(_Base):
    """One rank of a multi-GPU solve (RCCL).  `pg` is a torch.distributed process group used only
    for set-up (RCCL id broadcast, ghost lists); the solve itself never touches torch."""

    def __init__(self, G_data, Gc, keep_cols, n_full, rank, nranks, device, pg=None, structured=True):
        if nranks > 1:
            import torch.distributed as tdist
        self.L = load()
        self._setup_common(G_data, Gc, keep_cols, n_full, nranks)
        self.rank, self.nranks = rank, nranks
        self.structured = structured
        uid = np.zeros(128, np.uint8)
        if rank == 0 and self.L.lsq_dist_unique_id(ptr(uid)) != 0:
            raise NativeError('lsq_dist_unique_id failed')
        if nranks > 1:
            box = [uid.tobytes()]
            tdist.broadcast_object_list(box, src=0, group=pg)
            uid = np.frombuffer(box[0], np.uint8).copy()
        self.h = _quiet_stdout(lambda: self.L.lsq_create_dist(int(device), int(rank), int(nranks), ptr(uid)))
        if not self.h:
            raise NativeError('lsq_create_dist failed (RCCL communicator)')
        if structured:   # window of node rows on sub-grids, structured stencil operator
            self.prob = window_problem(G_data, Gc, self.partition, rank, keep_cols)
            _form_window(self.L, self.h, self.prob)
            _install_halo(self.L, self.h, self.prob,
                          window_halo(self.prob['grid_objs'], self.partition, rank, self.prob['halo']))
            self.has_blocks = _install_blocks(self.L, self.h, self.prob, keep_cols)
            self.has_global = _install_global(self.L, self.h, self.prob)
            self.n_x = self.prob['keep'].size
        else:            # owned rows, relabelled compact columns, assembled SELL operator
            self.prob = rank_problem(G_data, Gc, self.partition, rank)
            flags = _form_rank(self.L, self.h, self.prob, keep_cols, n_full)
            owner = column_owner(keep_cols, self.prob['grid_objs'], self.partition)
            self.layout = local_layout(flags, owner, rank)
            gathered = [self.layout[3]]
            if nranks > 1:
                gathered = [None] * nranks
                tdist.all_gather_object(gathered, self.layout[3], group=pg)
            self.plan = exchange_plan(rank, self.layout[0], gathered)
            _install_layout(self.L, self.h, self.layout, self.plan)
            self.owned_cols = self.layout[4]
            self.n_x = self.layout[2]
            self.has_blocks = False
        self.stats = None

    def scatter_owned(self, x_local, x_out):
        """Owned columns of this rank's solution into the global compact vector x_out."""
        if self.structured:
            window_owned_solution(self.prob, x_local, x_out)
        else:
            x_out[self.owned_cols] = x_local

    def _b(self, row_weight, rhs):
        """None keeps the weights / local rhs of the previous call (no host slicing)."""
        if row_weight is not None:
            self.set_row_weight(row_weight)
        if rhs is not None:
            self._b_local = as_c(np.asarray(rhs)[self.prob['rows']], np.float64)
        return self._b_local

    def set_row_weight(self, w):
        wl = as_c(np.asarray(w)[self.prob['rows']], np.float64)
        _HandleView(self.L, self.h).check(self.L.lsq_set_row_weight(self.h, ptr(wl)), 'lsq_set_row_weight')

    def solve(self, row_weight, rhs, atol=1e-10, btol=1e-10, conlim=1e8, maxit=0, precond=1, method=0):
        """method 0: LSQR (precond 0/1); 1: CGNR (precond 1 Jacobi, 3 block-Jacobi, 4 multigrid; structured
        ranks)."""
        b = self._b(row_weight, rhs)
        x = np.zeros(self.n_x)
        o = default_opts(atol=atol, btol=btol, conlim=conlim, maxit=int(maxit), precond=int(precond), method=int(method))
        st = LsqStats()
        _HandleView(self.L, self.h).check(self.L.lsq_solve(self.h, ptr(b), ptr(x), ctypes.byref(o), ctypes.byref(st)),
                                          'lsq_solve')
        self.stats = st.as_dict()
        return x   # this rank's columns: scatter_owned() places them in the global vector

    def iterate(self, row_weight, rhs, iters, precond=1, method=0):
        b = self._b(row_weight, rhs)
        o = default_opts(precond=int(precond), method=int(method))
        st = LsqStats()
        _HandleView(self.L, self.h).check(
            self.L.lsq_iterate(self.h, ptr(b), int(iters), ctypes.byref(o), ctypes.byref(st)), 'lsq_iterate')
        return st.as_dict()

    def info(self):
        o = np.zeros(8, np.int64)
        self.L.lsq_sell_info(self.h, ptr(o))
        return dict(zip(['m', 'n', 'nnz', 'sell_A', 'sell_AT', 'device_bytes', 'stencil_op', 'n_full'], o.tolist()))

    def comm_info(self):
        """What this rank's RCCL communicator and device report (lsq_dist_comm_info): comm_count,
        comm_rank, comm_device, device and the card's PCI id (domain:bus:device)."""
        o = np.zeros(7, np.int64)
        _HandleView(self.L, self.h).check(self.L.lsq_dist_comm_info(self.h, ptr(o)), 'lsq_dist_comm_info')
        return {'comm_count': int(o[0]), 'comm_rank': int(o[1]), 'comm_device': int(o[2]), 'device': int(o[3]),
                'pci': f'{int(o[4]):04x}:{int(o[5]):02x}:{int(o[6]):02x}'}

    def close(self):
        if getattr(self, 'h', None):
            self.L.lsq_destroy(self.h)
            self.h = None


class VirtualDistFitSystem(_Base):
    """All ranks of the partition in this process.  On one GPU (default; liblsqsurf virtual
    group): identical kernels, plans and exchange order as the RCCL path, exchanges are device
    copies.  With `devices` (distinct ids): liblsqsurf's device group, one RCCL communicator per
    device (ncclCommInitAll) and one host thread per rank during a solve."""

    def __init__(self, G_data, Gc, keep_cols, n_full, nranks, device=0, structured=True, devices=None):
        self.L = load()
        self._setup_common(G_data, Gc, keep_cols, n_full, nranks)
        self.nranks = nranks
        self.structured = structured
        if devices is not None:
            devs = as_c(np.asarray(devices, np.int32), np.int32)
            if devs.size != nranks or np.unique(devs).size != nranks:
                raise ValueError('a device group needs one distinct device per rank')
            self._api = 'lsq_dgroup'
            self.g = self.L.lsq_dgroup_create(int(nranks), ptr(devs))
        else:
            self._api = 'lsq_vgroup'
            self.g = self.L.lsq_vgroup_create(int(device), int(nranks))
        if not self.g:
            raise NativeError(f'{self._api}_create failed')
        self.probs = []
        self.has_blocks = self.has_global = structured
        if structured:
            for r in range(nranks):
                h = self._rank(r)
                prob = window_problem(G_data, Gc, self.partition, r, keep_cols)
                _form_window(self.L, h, prob)
                _install_halo(self.L, h, prob, window_halo(prob['grid_objs'], self.partition, r, prob['halo']))
                self.has_blocks &= _install_blocks(self.L, h, prob, keep_cols)
                self.has_global &= _install_global(self.L, h, prob)
                self.probs.append(prob)
            self.nx = [p['keep'].size for p in self.probs]
        else:
            if self._api == 'lsq_dgroup':
                raise NotImplementedError('device groups run structured ranks')
            flags_all = []
            for r in range(nranks):
                h = self._rank(r)
                prob = rank_problem(G_data, Gc, self.partition, r)
                flags_all.append(_form_rank(self.L, h, prob, keep_cols, n_full))
                self.probs.append(prob)
            owner = column_owner(keep_cols, self.probs[0]['grid_objs'], self.partition)
            self.layouts = [local_layout(flags_all[r], owner, r) for r in range(nranks)]
            ghosts_of = [lay[3] for lay in self.layouts]
            for r in range(nranks):
                _install_layout(self.L, self._rank(r), self.layouts[r], exchange_plan(r, self.layouts[r][0], ghosts_of))
            self.nx = [lay[2] for lay in self.layouts]
        self.stats = None

    def _fn(self, name):
        return getattr(self.L, f'{self._api}_{name}')

    def _rank(self, r):
        return self._fn('rank')(self.g, r)

    def _check(self, rc, what):
        if rc < 0:
            raise NativeError(f'{what}: {self._fn("last_error")(self.g).decode()}')

    def _bs(self, row_weight, rhs):
        if row_weight is not None:
            for r, prob in enumerate(self.probs):
                h = self._rank(r)
                wl = as_c(np.asarray(row_weight)[prob['rows']], np.float64)
                _HandleView(self.L, h).check(self.L.lsq_set_row_weight(h, ptr(wl)), 'lsq_set_row_weight')
        if rhs is not None:
            self._b_local = [as_c(np.asarray(rhs)[prob['rows']], np.float64) for prob in self.probs]
        return getattr(self, '_b_local', None)

    def set_row_mask(self, keep):
        """Rows kept in the solve (global row order; None: all)."""
        for r, prob in enumerate(self.probs):
            h = self._rank(r)
            k = None if keep is None else as_c(np.asarray(keep, bool)[prob['rows']], np.uint8)
            _HandleView(self.L, h).check(self.L.lsq_set_row_mask(h, ptr(k)), 'lsq_set_row_mask')

    def data_forward(self, x, n_data):
        """G_data · x for the global compact x (every data row on the rank that owns it)."""
        out = np.empty(int(n_data))
        for r, prob in enumerate(self.probs):
            h = self._rank(r)
            xl = as_c(np.asarray(x)[prob['keep_global']], np.float64)
            y = np.zeros(prob['npts'])
            _HandleView(self.L, h).check(self.L.lsq_spmv_rows(h, 0, prob['npts'], ptr(xl), ptr(y)), 'lsq_spmv_rows')
            out[prob['rows'][:prob['npts']]] = y
        return out

    def rows_sumsq(self, x, ranges):
        """lsq_rows_sumsq over the ranks: for each (first, count) range of GLOBAL rows, (Σ (w·G x)²,
        Σ (G x)²) — each stencil row lives on the rank that owns its centre, so the per-rank sums
        over the pieces of the range a rank holds add up to the single-GPU sums.  x: global compact.
        Stencil rows only (data rows: data_forward)."""
        if not self.structured:
            raise NotImplementedError('rows_sumsq over ranks needs structured ranks')
        sw, su = np.zeros(len(ranges)), np.zeros(len(ranges))
        for r, prob in enumerate(self.probs):
            pieces, which = [], []
            for i, (g0, cnt) in enumerate(ranges):
                for lrow0, first, n in prob['part_rows']:
                    a, b = max(g0, first), min(g0 + cnt, first + n)
                    if a < b:
                        pieces.append((lrow0 + a - first, b - a))
                        which.append(i)
            if not pieces:
                continue
            h = self._rank(r)
            xl = as_c(np.asarray(x)[prob['keep_global']], np.float64)
            f = as_c([p_[0] for p_ in pieces], np.int64)
            c = as_c([p_[1] for p_ in pieces], np.int64)
            a, b = np.zeros(len(pieces)), np.zeros(len(pieces))
            _HandleView(self.L, h).check(self.L.lsq_rows_sumsq(h, ptr(xl), len(pieces), ptr(f), ptr(c), ptr(a), ptr(b)),
                                         'lsq_rows_sumsq')
            np.add.at(sw, which, a)
            np.add.at(su, which, b)
        return sw, su

    def data_colsum(self, f, n_full):
        """G_dataᵀ f over the global full column space (f per global data row): every rank's
        node gather over its own points, summed into the global columns of its window."""
        out = np.zeros(int(n_full))
        f = np.asarray(f, np.float64)
        for r, prob in enumerate(self.probs):
            h = self._rank(r)
            fl = as_c(f[prob['rows'][:prob['npts']]], np.float64)
            loc = np.zeros(prob['n_full'])
            _HandleView(self.L, h).check(self.L.lsq_data_colsum(h, ptr(fl), ptr(loc)), 'lsq_data_colsum')
            out[prob['l2g']] += loc
        return out

    def solve(self, row_weight, rhs, atol=1e-10, btol=1e-10, conlim=1e8, maxit=0, precond=1, method=0, x0=None,
              anorm0=0.0):
        """x0 (global compact, CGNR on structured ranks): warm start; each rank starts from x0 on
        its window's columns.  anorm0 (CGNR): the stopping rule's starting ‖A‖ estimate
        (lsq_opts.anorm0; every rank runs the same scalar recurrence, so one value for all)."""
        bs = self._bs(row_weight, rhs)
        warm = x0 is not None and self.structured and int(method) == 1
        if warm:
            xs = [np.ascontiguousarray(np.asarray(x0, np.float64)[p['keep_global']]) for p in self.probs]
        else:
            xs = [np.zeros(k) for k in self.nx]
        bp = (ctypes.c_void_p * self.nranks)(*[b.ctypes.data for b in bs])
        xp = (ctypes.c_void_p * self.nranks)(*[x.ctypes.data for x in xs])
        o = default_opts(atol=atol, btol=btol, conlim=conlim, maxit=int(maxit), precond=int(precond), method=int(method),
                         use_x0=int(warm), anorm0=float(anorm0))
        st = LsqStats()
        self._check(self._fn('solve')(self.g, bp, xp, ctypes.byref(o), ctypes.byref(st)), f'{self._api}_solve')
        self.stats = st.as_dict()
        x = np.zeros(self.keep_cols.size)
        for r, xr in enumerate(xs):
            if self.structured:
                window_owned_solution(self.probs[r], xr, x)
            else:
                x[self.layouts[r][4]] = xr
        return x   # compact columns (same space as LSQSolver.solve)

    def iterate(self, row_weight, rhs, iters, precond=1, method=0):
        bs = self._bs(row_weight, rhs)
        bp = (ctypes.c_void_p * self.nranks)(*[b.ctypes.data for b in bs])
        o = default_opts(precond=int(precond), method=int(method))
        st = LsqStats()
        self._check(self._fn('iterate')(self.g, bp, int(iters), ctypes.byref(o), ctypes.byref(st)),
                    f'{self._api}_iterate')
        return st.as_dict()

    def close(self):
        if getattr(self, 'g', None):
            self._fn('destroy')(self.g)
            self.g = None


class MultiDeviceFitSystem:
    """smooth_fit's device system over several GPUs of this process (smooth_fit(n_gpus=N)): the
    y-slab ranks of a device group (distinct devices) or, for testing on one GPU, a virtual group.
    The FitSystem surface iterate_fit and parse_model use: solve with re-weighting, row editing
    and warm starts (CGNR), expand, data_forward, rows_sumsq, data_colsum — every product on the
    ranks' devices, so no host copy of the constraint operator is made.  compute_E forms its own
    single-device system (errors.py)."""
    formation = 'stencil'
    dense_ok = False        # no single-GPU dense factor over ranks

    def __init__(self, G_data, Gc, keep_cols, n_full, devices):
        self.n_data, self.n_con = int(G_data.N_eq), int(Gc.N_eq)
        self.keep_cols = np.asarray(keep_cols)
        self.n_full = int(n_full)
        devices = [int(d) for d in devices]
        same = len(set(devices)) == 1 and len(devices) > 1
        self.group = VirtualDistFitSystem(G_data, Gc, keep_cols, n_full, len(devices), device=devices[0],
                                          devices=None if same else devices)
        self.has_blocks = self.group.has_blocks
        self._mg = None
        self.mg_build_s = 0.0
        self.stats = None
        self._w_last = self._keep_last = self._rhs_last = None

    def multigrid_available(self, row_weight=None):
        """Multigrid over the ranks (precond 4) needs node blocks and the global description on
        every rank; its levels are built by the first solve (a failure there falls back)."""
        if self._mg is None:
            self._mg = bool(self.group.has_blocks and self.group.has_global)
        return self._mg

    def solve(self, row_weight, data_keep, rhs, x0=None, **opts):
        if row_weight is not self._w_last:
            self.group._bs(row_weight, None)
            self._w_last = row_weight
        dk = np.asarray(data_keep, dtype=bool)
        if self._keep_last is None or not np.array_equal(dk, self._keep_last):
            self.group.set_row_mask(np.concatenate([dk, np.ones(self.n_con, dtype=bool)]))
            self._keep_last = dk.copy()
        if opts.get('precond') in (0, 2, 5):   # single-GPU factorisations: the ranks' block-Jacobi instead
            opts = dict(opts, precond=3 if self.has_blocks else 1, method=1 if self.has_blocks else 0)
        if rhs is self._rhs_last:
            rhs = None                         # the ranks keep their slices
        else:
            self._rhs_last = rhs
        x = self.group.solve(None, rhs, x0=x0, **{k: v for k, v in opts.items()
                                                   if k in ('atol', 'btol', 'conlim', 'maxit', 'precond', 'method',
                                                            'anorm0')})
        self.stats = self.group.stats
        return x

    def expand(self, x):
        m0 = np.zeros(self.n_full)
        m0[self.keep_cols] = x
        return m0

    def data_forward(self, x):
        return self.group.data_forward(x, self.n_data)

    def rows_sumsq(self, x, ranges):
        return self.group.rows_sumsq(x, ranges)

    def data_colsum(self, f):
        return self.group.data_colsum(f, self.n_full)

    def close(self):
        self.group.close()


__all__ = ['SlabPartition', 'rank_problem', 'column_owner', 'local_layout', 'exchange_plan', 'DistFitSystem',
           'VirtualDistFitSystem', 'MultiDeviceFitSystem', 'LSQSolver']
