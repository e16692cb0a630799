"""Smoothness constraints and the reference-epoch column elimination.

Host mirror of LSsurf/constraint_functions.py:
  setup_smoothness_constraints  :23-109  — E_RMS keys -> constraint lin_ops with row sigma
      ``expected = E_RMS[key] / sqrt(prod(delta)) * mask_for_ind0(mask_scale)``
  build_reference_epoch_matrix  :112-151 — Ip_c, dropping dz[:, :, reference_epoch]
"""
import numpy as np
import scipy.sparse as sp

from .lin_op import lin_op


def _scaled(op, base, mask_scale, scaling_masks, keys):
    op.expected = op.mask_for_ind0(mask_scale)   # a fresh array: scaled in place (base · m, bitwise)
    op.expected *= base
    for key in keys:
        if key in scaling_masks:
            op.expected *= op.mask_for_ind0(mask=scaling_masks[key])
            break
    return op


def setup_smoothness_constraints(grids, constraint_op_list, E_RMS, mask_scale, scaling_masks=None):
    scaling_masks = scaling_masks or {}
    z0, dz = grids['z0'], grids['dz']
    root_A = np.sqrt(np.prod(z0.delta))
    if 'd2z0_dx2' in E_RMS:
        op = lin_op(z0, name='grad2_z0').grad2(DOF='z0')
        constraint_op_list.append(_scaled(op, E_RMS['d2z0_dx2'] / root_A, mask_scale, scaling_masks, ['d2z0_dx2']))
    if 'dz0_dx' in E_RMS:
        op = lin_op(z0, name='grad_z0').grad(DOF='z0')
        constraint_op_list.append(_scaled(op, E_RMS['dz0_dx'] / root_A, mask_scale, scaling_masks,
                                          ['dz0_dx', 'd2z0_dx2']))
    if E_RMS.get('z0') is not None:
        op = lin_op(z0, name='mag_z0').one(DOF='z0')
        op.expected = E_RMS['z0'] / root_A * np.ones_like(np.ravel(op.v))
        constraint_op_list.append(op)

    root_V = np.sqrt(np.prod(dz.delta))
    if E_RMS.get('d3z_dx2dt') is not None:
        op = lin_op(dz, name='grad2_dzdt').grad2_dzdt(DOF='z', t_lag=1)
        constraint_op_list.append(_scaled(op, E_RMS['d3z_dx2dt'] / root_V, mask_scale, scaling_masks, ['d3z_dx2dt']))
    if E_RMS.get('d2z_dxdt') is not None:
        op = lin_op(dz, name='grad_dzdt').grad_dzdt(DOF='z', t_lag=1)
        constraint_op_list.append(_scaled(op, E_RMS['d2z_dxdt'] / root_V, mask_scale, scaling_masks,
                                          ['d2z_dx2dt', 'd3z_dx2dt']))
    if E_RMS.get('d2z_dt2') is not None:
        op = lin_op(dz, name='d2z_dt2').d2z_dt2(DOF='z')
        op.expected = np.zeros(op.N_eq) + E_RMS['d2z_dt2'] / root_V
        if 'd2z_dt2' in scaling_masks:
            op.expected *= op.mask_for_ind0(mask=scaling_masks['d2z_dt2'])
        constraint_op_list.append(op)
    if 'dz' in scaling_masks:
        every = lin_op(dz, name='dz_zero').one(DOF='dz')
        e_dz = every.mask_for_ind0(mask=scaling_masks['dz'])
        sel = np.flatnonzero((e_dz > 0) & np.isfinite(e_dz))
        op = lin_op(dz, name='dz_zero').one(DOF='dz', which_nodes=sel + dz.col_0)
        op.expected = e_dz[sel]
        constraint_op_list.append(op)
    if E_RMS.get('lagrangian_dz') is not None:
        lg = grids['lagrangian_dz']
        root = np.sqrt(lg.delta[0] * lg.delta[1])
        op = lin_op(lg, name='lagrangian_rms').one(DOF='lagrangian_dz')
        op.expected = np.zeros(op.N_eq) + E_RMS['lagrangian_dz'] / root
        constraint_op_list.append(op)
    if E_RMS.get('lagrangian_dzdx') is not None:
        lg = grids['lagrangian_dz']
        root = np.sqrt(lg.delta[0] * lg.delta[1])
        op = lin_op(lg, name='lagrangian_rms_grad').grad(DOF='lagrangian_dz')
        op.expected = np.zeros(op.N_eq) + E_RMS['lagrangian_dzdx'] / root
        constraint_op_list.append(op)
    for op in constraint_op_list:
        if not np.all(op.expected):   # no boolean temporary of the op's rows
            raise ValueError(f'found zero value in the expected values for {op.name}')


def reference_epoch_keep_cols(n_cols, dz_grid, reference_epoch):
    """Columns kept by Ip_c: every column except dz[:, :, reference_epoch] (ascending; the
    np.setdiff1d of constraint_functions.py:112-151, as a boolean mask)."""
    iy, ix = np.meshgrid(np.arange(dz_grid.shape[0]), np.arange(dz_grid.shape[1]), indexing='ij')
    ref_cols = dz_grid.global_ind([iy.T.ravel(), ix.T.ravel(), np.full(iy.size, reference_epoch)])
    keep = np.ones(int(n_cols), dtype=bool)
    keep[ref_cols[(ref_cols >= 0) & (ref_cols < n_cols)]] = False
    return np.flatnonzero(keep).astype('int', copy=False)


def build_reference_epoch_matrix(G_data, Gc, grids, reference_epoch, dz_mask=None):
    if dz_mask is not None:
        raise NotImplementedError('build_reference_epoch_matrix: dz_mask is outside lssurf_amd')
    keep = reference_epoch_keep_cols(G_data.col_N, grids['dz'], reference_epoch)
    return sp.coo_matrix((np.ones_like(keep), (keep, np.arange(keep.size))), shape=(Gc.col_N, keep.size)).tocsc()


def _node_column_blocks_uniform(z0, dz, keep_cols, max_block):
    """node_column_blocks' usual case — the same kept columns at every node, one block per node
    (≤ max_block columns) — from views of the compact-position map (int32, no (nodes × k) index
    arrays): the same (block_ptr, cols); None when the case does not apply."""
    ny, nx, nt = (int(s) for s in dz.shape)
    nn = ny * nx
    same = z0 is not None and tuple(z0.shape) == (ny, nx) and all(
        np.array_equal(a, b) for a, b in zip(z0.ctrs, dz.ctrs[:2]))
    n_full = max(int(dz.col_0) + nn * nt, int(z0.col_0) + nn if same else 0,
                 int(keep_cols.max()) + 1 if keep_cols.size else 0)
    if n_full >= 2 ** 31 or keep_cols.size == 0:
        return None
    where = np.full(n_full, -1, dtype=np.int32)
    where[keep_cols] = np.arange(keep_cols.size, dtype=np.int32)
    wdz = where[int(dz.col_0):int(dz.col_0) + nn * nt].reshape(nn, nt)
    tkeep = wdz[0] >= 0
    if not np.array_equal(wdz >= 0, np.broadcast_to(tkeep, wdz.shape)):
        return None
    zk = False
    if same:
        wz = where[int(z0.col_0):int(z0.col_0) + nn]
        zk = bool(wz[0] >= 0)
        if not np.all((wz >= 0) == zk):
            return None
    k = int(tkeep.sum()) + (1 if zk else 0)
    if k == 0 or k > max_block:
        return None
    cols = np.empty((nn, k), dtype=np.int32)
    if zk:
        cols[:, 0] = wz
    cols[:, int(zk):] = wdz[:, tkeep]
    return np.arange(0, (nn + 1) * k, k, dtype=np.int64), cols.ravel()


def node_column_blocks_affine(grids, keep_cols, max_block=16):
    """node_column_blocks' usual case as its affine structure, for lsq_set_column_blocks_affine:
    (n_blocks, base, stride, full_base, full_stride) with block b = the compact columns
    base[j] + b·stride[j] (full ids full_base[j] + b·full_stride[j]) — the same blocks, in the same
    order, as node_column_blocks.  Read from nodes 0 and 1 only (binary searches in the ascending
    keep_cols); the library checks every node on the device.  None when the structure does not
    apply (then node_column_blocks)."""
    z0, dz = grids.get('z0'), grids.get('dz')
    if dz is None or dz.N_dims != 3:
        return None
    keep_cols = np.asarray(keep_cols)
    ny, nx, nt = (int(s) for s in dz.shape)
    nn = ny * nx
    if nn < 2 or keep_cols.size == 0:
        return None
    same = z0 is not None and tuple(z0.shape) == (ny, nx) and all(
        np.array_equal(a, b) for a, b in zip(z0.ctrs, dz.ctrs[:2]))
    fstride = ([1] if same else []) + [nt] * nt
    full0 = np.array(([int(z0.col_0)] if same else []) + [int(dz.col_0) + t for t in range(nt)], dtype=np.int64)
    full1 = full0 + np.array(fstride, dtype=np.int64)
    pos0, pos1 = np.searchsorted(keep_cols, full0), np.searchsorted(keep_cols, full1)
    kept0 = (pos0 < keep_cols.size) & (keep_cols[np.minimum(pos0, keep_cols.size - 1)] == full0)
    kept1 = (pos1 < keep_cols.size) & (keep_cols[np.minimum(pos1, keep_cols.size - 1)] == full1)
    k = int(kept0.sum())
    if not np.array_equal(kept0, kept1) or k == 0 or k > max_block or nn * k != keep_cols.size:
        return None
    base = pos0[kept0].astype(np.int64)
    return (nn, base, pos1[kept0].astype(np.int64) - base, full0[kept0],
            np.array(fstride, dtype=np.int64)[kept0])


def node_column_blocks(grids, keep_cols, max_block=16):
    """Column blocks of the block-Jacobi preconditioner (lsq precond 3):
    one block per (y, x) node = its z0 column (when the z0 and dz grids share the node lattice)
    and its dz columns of every kept epoch, in compact column ids (`keep_cols` ascending, as
    returned by reference_epoch_keep_cols).  Blocks longer than `max_block` are split along t.
    Returns (block_ptr, cols) or None when the grids do not have that structure."""
    z0, dz = grids.get('z0'), grids.get('dz')
    if dz is None or dz.N_dims != 3:
        return None
    keep_cols = np.asarray(keep_cols)
    ny, nx, nt = (int(s) for s in dz.shape)
    fast = _node_column_blocks_uniform(z0, dz, keep_cols, max_block)
    if fast is not None:
        return fast
    nodes = np.arange(ny * nx)
    dz_cols = dz.col_0 + nodes[:, None] * nt + np.arange(nt)[None, :]          # (nodes, nt) full ids
    same = z0 is not None and tuple(z0.shape) == (ny, nx) and all(
        np.array_equal(a, b) for a, b in zip(z0.ctrs, dz.ctrs[:2]))
    parts = [(z0.col_0 + nodes)[:, None]] if same else []
    full = np.concatenate(parts + [dz_cols], axis=1)                           # (nodes, k)
    # compact position of every full column (a scatter, not a sorted search: keep_cols ascending)
    n_full = int(max(full.max(), keep_cols.max() if keep_cols.size else 0)) + 1
    where = np.full(n_full, -1, dtype=np.int64)
    where[keep_cols] = np.arange(keep_cols.size)
    pos = where[full]
    kept = pos >= 0
    pos_c = np.where(kept, pos, 0)
    cols, lens = [], []
    k_all = kept.sum(axis=1)
    if np.all(k_all == k_all[0]):                 # the usual case: same kept set at every node
        k = int(k_all[0])
        comp = pos_c[kept].reshape(-1, k)
        nsplit = -(-k // max_block)
        for s in range(nsplit):
            sl = comp[:, s * max_block:(s + 1) * max_block]
            cols.append(sl)
            lens.append(np.full(sl.shape[0], sl.shape[1]))
        order = np.argsort(np.concatenate([np.arange(ny * nx) * nsplit + s for s in range(nsplit)]), kind='stable')
        lens = np.concatenate(lens)[order]
        flat = np.concatenate([c.reshape(-1, c.shape[1]) for c in cols]) if nsplit == 1 else None
        if nsplit == 1:
            cols = flat.ravel()
        else:
            rows = [list(c) for c in cols]
            cols = np.concatenate([np.concatenate([rows[s][i] for s in range(nsplit)]) for i in range(ny * nx)])
    else:
        out = [pos_c[i][kept[i]] for i in range(ny * nx)]
        chunks = [o[s:s + max_block] for o in out for s in range(0, max(len(o), 1), max_block) if len(o)]
        lens = np.array([len(c) for c in chunks])
        cols = np.concatenate(chunks)
    ptr = np.r_[0, np.cumsum(lens)].astype(np.int64)
    return ptr, np.asarray(cols, dtype=np.int32)
