"""Host mirror of the solve boundary: a handle on one MI355X holding the formed least-squares
system, plus drop-ins for the reference's Cython triangular kernels.

* ``LSQSolver``  — replaces ``sparseqr.solve`` (LSsurf/smooth_fit.py:142) and the residual
  products ``G_data.toCSR().dot(m0)`` (smooth_fit.py:146,662).  The COO triplets of the
  unweighted operator, the column map Ip_c, the row weights (TCinv) and the row selection Ip_r
  go to the device once; outer iterations only change weights / masks.
* ``inv_tr_upper``, ``propagate_qz_errors``, ``spsolve_tr_upper`` — same signatures and
  outputs as LSsurf/inv_tr_upper.pyx:19, propagate_qz_errors.pyx:15, spsolve_tr_upper.pyx:11,
  computed by liblsqsurf's HIP kernels.
"""
import ctypes

import numpy as np
import scipy.sparse as sp

from ._native import LsqStats, NativeError, NativeRefused, as_c, default_opts, load, ptr


class LSQSolver:
    """One device-resident least-squares system ``min || diag(w)·mask·(G x − b) ||``."""

    def __init__(self, device=0):
        self._L = load()
        self._h = self._L.lsq_create(int(device))
        if not self._h:
            raise NativeError(f'lsq_create({device}) failed: no gfx950 (MI355X) device visible')
        self.device = device
        self.m = self.n = self.n_full = None

    # ---- lifetime --------------------------------------------------------------------------
    def close(self):
        if getattr(self, '_h', None):
            self._L.lsq_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc, what):
        if rc < 0:
            cls = NativeRefused if rc == -5 else NativeError
            raise cls(f'{what}: {self._L.lsq_last_error(self._h).decode()}')
        return rc

    # ---- formation ---------------------------------------------------------------------------
    def set_col_map(self, n_full, keep_cols):
        keep = as_c(keep_cols, np.int64)
        self._check(self._L.lsq_set_col_map(self._h, int(n_full), ptr(keep), keep.size), 'lsq_set_col_map')
        self.n = keep.size
        self.n_full = int(n_full)

    def set_matrix_coo(self, m, n_full, r, c, v, row_weight=None):
        r, c, v = as_c(r, np.int64).ravel(), as_c(c, np.int64).ravel(), as_c(v, np.float64).ravel()
        w = None if row_weight is None else as_c(row_weight, np.float64)
        self._check(self._L.lsq_set_matrix_coo(self._h, int(m), int(n_full), v.size, ptr(r), ptr(c), ptr(v), ptr(w)),
                    'lsq_set_matrix_coo')
        self.m = int(m)
        if self.n is None:
            self.n = int(n_full)
        self.n_full = int(n_full)

    def set_matrix_stencil(self, m, n_full, grids, interp_grid, coords, stencils, npts, row_weight=None, fields=()):
        """Structured formation (lssurf_amd.assemble.describe output) — rows generated on device.
        fields: field-valued parts [(stencil index, off (ntpl×3), val, fsel, F (nfield × n_eq))]."""
        from ._native import GridDesc, StencilDesc
        for k, off, val, fsel, F in fields:
            off, val = as_c(off, np.int32).reshape(-1, 3), as_c(val, np.float64)
            fsel, F = as_c(fsel, np.int32), as_c(F, np.float64)
            self._check(self._L.lsq_set_stencil_fields(self._h, int(k), off.shape[0], ptr(off), ptr(val), F.shape[0],
                                                       ptr(fsel), F.shape[1], ptr(F)), 'lsq_set_stencil_fields')
        ga = (GridDesc * len(grids))(*grids)
        sa = (StencilDesc * max(len(stencils), 1))(*stencils)
        ig = as_c(np.asarray(interp_grid, dtype=np.int32), np.int32)
        py, px, pt = coords
        w = None if row_weight is None else as_c(row_weight, np.float64)
        self._check(self._L.lsq_set_matrix_stencil(self._h, int(m), int(n_full), len(grids), ctypes.cast(ga, ctypes.c_void_p),
                                                   len(interp_grid), ptr(ig), int(npts), ptr(py), ptr(px), ptr(pt),
                                                   len(stencils), ctypes.cast(sa, ctypes.c_void_p), ptr(w)),
                    'lsq_set_matrix_stencil')
        self.m = int(m)
        if self.n is None:
            self.n = int(n_full)
        self.n_full = int(n_full)

    def set_row_weight(self, w):
        w = None if w is None else as_c(w, np.float64)
        self._check(self._L.lsq_set_row_weight(self._h, ptr(w)), 'lsq_set_row_weight')

    def set_row_mask(self, keep):
        # a bool array is passed as its bytes (0/1: no copy); any non-zero byte keeps the row
        k = None if keep is None else (keep.view(np.uint8) if isinstance(keep, np.ndarray) and keep.dtype == bool
                                       and keep.flags.c_contiguous else as_c(np.asarray(keep, dtype=bool), np.uint8))
        self._check(self._L.lsq_set_row_mask(self._h, ptr(k)), 'lsq_set_row_mask')

    def set_column_blocks(self, blocks):
        """Column blocks of the block-Jacobi preconditioner (precond 3): a list of compact-column
        index arrays (≤ 16 columns each); unlisted columns become singletons.  None clears."""
        if not blocks:
            self._check(self._L.lsq_set_column_blocks(self._h, 0, None, None), 'lsq_set_column_blocks')
            return
        ptr_ = as_c(np.r_[0, np.cumsum([len(b) for b in blocks])], np.int64)
        cols = as_c(np.concatenate([np.asarray(b) for b in blocks]), np.int32)
        self._check(self._L.lsq_set_column_blocks(self._h, len(blocks), ptr(ptr_), ptr(cols)),
                    'lsq_set_column_blocks')

    def set_column_blocks_csr(self, block_ptr, cols):
        """Same as set_column_blocks with the blocks given as (block_ptr, cols) arrays."""
        p_ = as_c(block_ptr, np.int64)
        c_ = as_c(cols, np.int32)
        self._check(self._L.lsq_set_column_blocks(self._h, p_.size - 1, ptr(p_), ptr(c_)), 'lsq_set_column_blocks')

    def set_column_blocks_affine(self, n_blocks, base, stride, full_base, full_stride):
        """Blocks b < n_blocks of the compact columns base[j] + b·stride[j] with full ids
        full_base[j] + b·full_stride[j] (lsq_set_column_blocks_affine: formed and checked on the
        device; NativeError when the structure does not hold)."""
        a = [as_c(np.asarray(v, dtype=np.int64), np.int64) for v in (base, stride, full_base, full_stride)]
        self._check(self._L.lsq_set_column_blocks_affine(self._h, int(n_blocks), a[0].size, *(ptr(v) for v in a)),
                    'lsq_set_column_blocks_affine')

    def shape(self):
        m, n, z = (ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64())
        self._check(self._L.lsq_shape(self._h, ctypes.byref(m), ctypes.byref(n), ctypes.byref(z)), 'lsq_shape')
        return m.value, n.value, z.value

    def get_csr(self):
        """The formed A = Ip_r·TCinv·G·Ip_c (selected rows), as scipy CSR."""
        m, n, z = self.shape()
        rp = np.zeros(m + 1, np.int64)
        ci = np.zeros(max(z, 1), np.int32)
        v = np.zeros(max(z, 1))
        self._check(self._L.lsq_get_csr(self._h, ptr(rp), ptr(ci), ptr(v)), 'lsq_get_csr')
        return sp.csr_matrix((v[:z], ci[:z], rp), shape=(m, n))

    def release_full_csr(self):
        """Free the full G / Gᵀ (and SELL copies) that lsq_get_csr, the dense / band factors or
        lsq_spmv formed on a lazily formed structured system; True when something was freed."""
        r = ctypes.c_int32()
        self._check(self._L.lsq_release_full_csr(self._h, ctypes.byref(r)), 'lsq_release_full_csr')
        return bool(r.value)

    # ---- solve -------------------------------------------------------------------------------
    def solve(self, b, x0=None, atol=1e-10, btol=1e-10, conlim=1e8, maxit=0, precond=1, batch=0,
              use_graph=True, op=0, method=0, b_rows=0, anorm0=0.0):
        """LSQR (method 0) or CGNR (method 1: PCG on the normal equations with the fused
        normal-stencil operator; LSQR where that operator does not exist — stats['method'] says
        which ran); returns (x, stats) with scipy-lsqr-style stats (iters, istop, r1norm, ...).
        precond: 1 Jacobi, 2 dense Cholesky, 3 block-Jacobi per node, 4 multigrid V-cycle (CGNR
        only).  batch 0: the library's default iterations per host convergence check.  b_rows > 0:
        the caller guarantees b[b_rows:] == 0, so only b[:b_rows] crosses PCIe (smooth_fit: the
        data rows; the 73 M constraint rows of C4 are zero).  anorm0 (CGNR): stats['anorm'] of an
        earlier solve of the same operator and preconditioner — the stopping rule starts from it
        instead of rebuilding its ‖A‖ estimate (lsq_opts.anorm0)."""
        b = as_c(b, np.float64)
        if b.size != self.m:
            raise ValueError(f'b has {b.size} rows, system has {self.m}')
        x = np.zeros(self.n) if x0 is None else as_c(x0, np.float64).copy()
        o = default_opts(atol=atol, btol=btol, conlim=conlim, maxit=int(maxit), precond=int(precond),
                         use_x0=int(x0 is not None), batch=int(batch), use_graph=int(bool(use_graph)), op=int(op),
                         method=int(method), b_rows=int(b_rows), anorm0=float(anorm0))
        st = LsqStats()
        self._check(self._L.lsq_solve(self._h, ptr(b), ptr(x), ctypes.byref(o), ctypes.byref(st)), 'lsq_solve')
        return x, st.as_dict()

    def iterate(self, b, iters, precond=1, batch=0, use_graph=True, op=0, method=0, b_rows=0):
        b = as_c(b, np.float64)
        o = default_opts(precond=int(precond), batch=int(batch), use_graph=int(bool(use_graph)), op=int(op),
                         method=int(method), b_rows=int(b_rows))
        st = LsqStats()
        self._check(self._L.lsq_iterate(self._h, ptr(b), int(iters), ctypes.byref(o), ctypes.byref(st)),
                    'lsq_iterate')
        return st.as_dict()

    def profile_kernels(self, reps=20, op=0):
        """Per-kernel device time (ms) of one iteration's launches of operator `op`, and the
        algorithmic HBM bytes per launch of the two streaming kernels."""
        o = np.zeros(8)
        self._check(self._L.lsq_profile_kernels(self._h, int(reps), int(op), ptr(o)), 'lsq_profile_kernels')
        d = dict(zip(['xw_spmv', 'spmtv', 'beta', 'givens'], o[:4].tolist()))
        d['bytes'] = {'xw_spmv': float(o[4]), 'spmtv': float(o[5])}
        return d

    def cg_available(self, precond=3):
        """(True, '') when method 1 runs CGNR on this system with this preconditioner, else
        (False, reason) — method 1 then falls back to LSQR."""
        rc = self._check(self._L.lsq_cg_available(self._h, int(precond)), 'lsq_cg_available')
        return bool(rc), ('' if rc else self._L.lsq_last_error(self._h).decode())

    def profile_cg(self, reps=20, precond=3):
        """Per-kernel device time (ms) of one CGNR iteration and algorithmic bytes per launch."""
        o = np.zeros(8)
        self._check(self._L.lsq_profile_cg(self._h, int(reps), int(precond), ptr(o)), 'lsq_profile_cg')
        d = dict(zip(['cg_data', 'cg_normal', 'cg_update', 'cg_scalars'], o[:4].tolist()))
        d['bytes'] = {'cg_data': float(o[4]), 'cg_normal': float(o[5]), 'cg_update': float(o[6])}
        d['data_rows'] = 'matrix-free' if int(o[7]) & 1 else 'stored'
        d['normal_kernel'] = 'wave-strip' if int(o[7]) & 2 else 'ring'
        return d

    def mg_info(self):
        """Multigrid (precond 4) levels: list of (S0, S1, n_full) per level, and the removed epoch."""
        o = np.zeros(1 + 4 * 32, np.int64)
        self._check(self._L.lsq_mg_info(self._h, ptr(o), o.size), 'lsq_mg_info')
        L = int(o[0])
        self._mg_tail = int(o[1 + 4 * L])
        return [tuple(int(v) for v in o[1 + 4 * l:4 + 4 * l]) for l in range(L)], int(o[4])

    def mg_tail_level(self):
        """First level of the multigrid's one-workgroup tail V-cycle (k_mg_tail), −1 for none."""
        self.mg_info()
        return self._mg_tail

    def mg_apply(self, level, what, x=None):
        """Multigrid test hook: what 0 → N_l x on level l's full column space; 1 → V-cycle(x)
        (level 0); 2 → the smoother's λ_max(M⁻¹N) estimate of level l."""
        levels, _ = self.mg_info()
        nf = levels[level][2]
        if what == 2:
            y = np.zeros(1)
            self._check(self._L.lsq_mg_apply(self._h, int(level), 2, None, ptr(y)), 'lsq_mg_apply')
            return float(y[0])
        xx = as_c(x, np.float64)
        if xx.size != nf:
            raise ValueError(f'x must have {nf} entries')
        y = np.zeros(nf)
        self._check(self._L.lsq_mg_apply(self._h, int(level), int(what), ptr(xx), ptr(y)), 'lsq_mg_apply')
        return y

    def normal_apply(self, p_full):
        """q = AᵀA p over the full column space (current weights / mask)."""
        p = as_c(p_full, np.float64)
        if p.size != self.n_full:
            raise ValueError('p must have n_full entries')
        q = np.zeros(self.n_full)
        self._check(self._L.lsq_normal_apply(self._h, ptr(p), ptr(q)), 'lsq_normal_apply')
        return q

    def info(self):
        o = np.zeros(8, np.int64)
        self._check(self._L.lsq_sell_info(self._h, ptr(o)), 'lsq_sell_info')
        return dict(zip(['m', 'n', 'nnz', 'sell_A', 'sell_AT', 'device_bytes', 'stencil_op', 'n_full'], o.tolist()))

    def sigma_x(self):
        """sqrt(diag((AᵀA)⁻¹)) of the current weighted, masked system (dense device Cholesky)."""
        E = np.zeros(self.n)
        self._check(self._L.lsq_sigma_x(self._h, ptr(E)), 'lsq_sigma_x')
        return E

    def rinv(self):
        """R⁻¹ (n x n upper triangular, AᵀA = RᵀR) of the current weighted, masked system."""
        Ri = np.zeros((self.n, self.n))
        self._check(self._L.lsq_get_rinv(self._h, ptr(Ri)), 'lsq_get_rinv')
        return Ri

    def set_band_order(self, perm=None):
        """Column order for precond 5 (new position -> compact column; None = natural)."""
        pp = None if perm is None else as_c(perm, np.int32)
        n = 0 if pp is None else pp.size
        self._check(self._L.lsq_set_band_order(self._h, n, ptr(pp) if pp is not None else None),
                    'lsq_set_band_order')

    def band_factor(self, perm=None):
        """(R, perm): (A·P)ᵀ(A·P) = RᵀR for the current weighted, masked A, R upper triangular
        (scipy CSR, n × n, explicit zeros of the band dropped), P = perm (new position -> compact
        column) — the R and E of sparseqr.rz (lsq_band_factor)."""
        pp = None if perm is None else as_c(perm, np.int32)
        info = np.zeros(3, np.int64)
        self._check(self._L.lsq_band_factor(self._h, ptr(pp) if pp is not None else None, ptr(info), None, None, None),
                    'lsq_band_factor')
        n, T, w = (int(v) for v in info)
        R = np.zeros(T * (w + 1) * 4096)
        sc = np.zeros(T * 64)
        po = np.zeros(n, np.int32)
        self._check(self._L.lsq_band_factor(self._h, ptr(pp) if pp is not None else None, ptr(info), ptr(R), ptr(sc),
                                            ptr(po)), 'lsq_band_factor')
        tiles = R.reshape(T, w + 1, 64, 64)
        rows, cols, vals = [], [], []
        r64, c64 = np.meshgrid(np.arange(64), np.arange(64), indexing='ij')
        for I in range(T):
            for k in range(min(w + 1, T - I)):
                t = tiles[I, k]
                sel = (t != 0) & ((r64 <= c64) if k == 0 else True)
                rows.append(64 * I + r64[sel])
                cols.append(64 * (I + k) + c64[sel])
                vals.append(t[sel])
        rows, cols, vals = np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)
        keep = (rows < n) & (cols < n)
        vals = vals[keep] / sc[cols[keep]]            # R = R̃ S⁻¹ (column j scaled by 1/s_j)
        Rm = sp.csr_matrix((vals, (rows[keep], cols[keep])), shape=(n, n))
        Rm.sort_indices()
        return Rm, po

    def cov_band(self, perm=None, op=None):
        """(E, op_err, info) of the current weighted, masked system without a dense factor:
        E = sqrt(diag((AᵀA)⁻¹)) per compact column and, for the rows of `op` (scipy sparse over
        the compact columns), sqrt(diag(op (AᵀA)⁻¹ opᵀ)).  `perm` (new position -> compact column)
        should make AᵀA banded (lsq_cov_band)."""
        E = np.zeros(self.n)
        info = np.zeros(6, np.int64)
        pp = None if perm is None else as_c(perm, np.int32)
        if pp is not None and pp.size != self.n:
            raise ValueError('cov_band: perm must have one entry per column')
        if op is None:
            self._check(self._L.lsq_cov_band(self._h, ptr(pp) if pp is not None else None, ptr(E), 0, None, None,
                                             None, None, ptr(info)), 'lsq_cov_band')
            return E, None, info
        op = sp.csr_matrix(op)
        op.sort_indices()
        rp, ci, v = as_c(op.indptr, np.int64), as_c(op.indices, np.int32), as_c(op.data, np.float64)
        out = np.zeros(op.shape[0])
        self._check(self._L.lsq_cov_band(self._h, ptr(pp) if pp is not None else None, ptr(E), op.shape[0],
                                         ptr(rp), ptr(ci), ptr(v), ptr(out), ptr(info)), 'lsq_cov_band')
        return E, out, info

    def cov_band_window(self, perm_w, op=None, inner=None):
        """cov_band for a window W of the columns (perm_w: its compact columns in a banded order):
        E[j] = sqrt(((A_WᵀA_W)⁻¹)_jj) in WINDOW order (len(perm_w) entries) and the op rows' errors,
        every op row inside W (lsq_cov_band_window).  inner (bool per window position, None = all):
        only the tiles holding those positions are swept; E is 0 elsewhere."""
        pp = as_c(perm_w, np.int32)
        E = np.zeros(pp.size)
        info = np.zeros(6, np.int64)
        ii = None if inner is None else as_c(np.asarray(inner, dtype=bool), np.uint8)
        if ii is not None and ii.size != pp.size:
            raise ValueError('cov_band_window: inner must have one flag per window position')
        if op is None or op.shape[0] == 0:
            self._check(self._L.lsq_cov_band_window(self._h, ptr(pp), pp.size, ptr(ii), ptr(E), 0, None, None, None,
                                                    None, ptr(info)), 'lsq_cov_band_window')
            return E, np.zeros(0), info
        op = sp.csr_matrix(op)
        op.sort_indices()
        rp, ci, v = as_c(op.indptr, np.int64), as_c(op.indices, np.int32), as_c(op.data, np.float64)
        out = np.zeros(op.shape[0])
        self._check(self._L.lsq_cov_band_window(self._h, ptr(pp), pp.size, ptr(ii), ptr(E), op.shape[0], ptr(rp),
                                                ptr(ci), ptr(v), ptr(out), ptr(info)), 'lsq_cov_band_window')
        return E, out, info

    def cov_band_windows(self, windows):
        """cov_band_window for many windows at once, pipelined on the device (lsq_cov_band_windows):
        windows = [(perm_w, inner or None, op or None)] with op rows over the COMPACT columns, every
        row inside its window.  Returns ([E_w (window order)], [op_err_w or None], info)."""
        sizes = [len(w[0]) for w in windows]
        wp = as_c(np.r_[0, np.cumsum(sizes)], np.int64)
        perm = as_c(np.concatenate([np.asarray(w[0]) for w in windows]), np.int32)
        inner = as_c(np.concatenate([np.ones(sz, bool) if w[1] is None else np.asarray(w[1], bool)
                                     for w, sz in zip(windows, sizes)]), np.uint8)
        E = np.zeros(perm.size)
        info = np.zeros(6, np.int64)
        ops = [w[2] for w in windows]
        if all(o is None or o.shape[0] == 0 for o in ops):
            self._check(self._L.lsq_cov_band_windows(self._h, len(windows), ptr(wp), ptr(perm), ptr(inner), ptr(E),
                                                     None, None, None, None, None, ptr(info)), 'lsq_cov_band_windows')
            return [E[wp[i]:wp[i + 1]] for i in range(len(windows))], [None] * len(windows), info
        nrow = [0 if o is None else o.shape[0] for o in ops]
        wo = as_c(np.r_[0, np.cumsum(nrow)], np.int64)
        rps, poss, vals = [np.zeros(1, np.int64)], [], []
        base = 0
        pos_of = np.full(self.n, -1, np.int64)
        for (cols, _, op), nr in zip(windows, nrow):
            if not nr:
                continue
            op = sp.csr_matrix(op)
            op.sort_indices()
            pos_of[np.asarray(cols)] = np.arange(len(cols))
            p = pos_of[op.indices]
            pos_of[np.asarray(cols)] = -1
            if p.size and p.min() < 0:
                raise ValueError('cov_band_windows: an op row reaches outside its window')
            rps.append(op.indptr[1:].astype(np.int64) + base)
            base += op.indptr[-1]
            poss.append(p)
            vals.append(op.data)
        rp = as_c(np.concatenate(rps), np.int64)
        pos = as_c(np.concatenate(poss) if poss else np.zeros(0), np.int32)
        val = as_c(np.concatenate(vals) if vals else np.zeros(0), np.float64)
        oe = np.zeros(int(wo[-1]))
        self._check(self._L.lsq_cov_band_windows(self._h, len(windows), ptr(wp), ptr(perm), ptr(inner), ptr(E),
                                                 ptr(wo), ptr(rp), ptr(pos), ptr(val), ptr(oe), ptr(info)),
                    'lsq_cov_band_windows')
        return ([E[wp[i]:wp[i + 1]] for i in range(len(windows))],
                [oe[wo[i]:wo[i + 1]] if nrow[i] else None for i in range(len(windows))], info)

    def cov_band_windows_schur(self, windows):
        """cov_band_windows with each window's bottom margin eliminated first
        (lsq_cov_band_windows_schur): windows = [(perm_A, inner_A, perm_B or None, nib)], perm_A =
        [top margin, interior] rows ascending ending with the nib columns of Ib, perm_B = the band
        order of [Ib, bottom margin] reversed.  Returns ([E_w over perm_A], info)."""
        sa = [len(w[0]) for w in windows]
        sb = [0 if w[2] is None else len(w[2]) for w in windows]
        wp = as_c(np.r_[0, np.cumsum(sa)], np.int64)
        bp = as_c(np.r_[0, np.cumsum(sb)], np.int64)
        perm = as_c(np.concatenate([np.asarray(w[0]) for w in windows]), np.int32)
        inner = as_c(np.concatenate([np.ones(n, bool) if w[1] is None else np.asarray(w[1], bool)
                                     for w, n in zip(windows, sa)]), np.uint8)
        bperm = as_c(np.concatenate([np.asarray(w[2]) for w in windows if w[2] is not None] or [np.zeros(0)]),
                     np.int32)
        nib = as_c(np.array([w[3] if w[2] is not None else 0 for w in windows]), np.int64)
        E = np.zeros(perm.size)
        info = np.zeros(6, np.int64)
        self._check(self._L.lsq_cov_band_windows_schur(self._h, len(windows), ptr(wp), ptr(perm), ptr(inner), ptr(E),
                                                       ptr(bp), ptr(bperm), ptr(nib), ptr(info)),
                    'lsq_cov_band_windows_schur')
        return [E[wp[i]:wp[i + 1]] for i in range(len(windows))], info

    def spmv(self, x, trans=False):
        """G x (trans False) or Gᵀ x on the UNWEIGHTED formed operator, all rows."""
        x = as_c(x, np.float64)
        nout = self.n if trans else self.m
        y = np.zeros(nout)
        self._check(self._L.lsq_spmv(self._h, int(bool(trans)), ptr(x), ptr(y)), 'lsq_spmv')
        return y


    def rows_sumsq(self, x, ranges):
        """For each (first, count) row range: (Σ (w_i (G x)_i)², Σ (G x)_i²), w = row weights."""
        x = as_c(x, np.float64)
        f = as_c([r[0] for r in ranges], np.int64)
        c = as_c([r[1] for r in ranges], np.int64)
        sw, su = np.zeros(len(ranges)), np.zeros(len(ranges))
        self._check(self._L.lsq_rows_sumsq(self._h, ptr(x), len(ranges), ptr(f), ptr(c), ptr(sw), ptr(su)),
                    'lsq_rows_sumsq')
        return sw, su

    def data_colsum(self, f):
        """G_dataᵀ f over the full column space (unweighted data rows; f per data row)."""
        f = as_c(f, np.float64)
        out = np.zeros(self.n_full)
        self._check(self._L.lsq_data_colsum(self._h, ptr(f), ptr(out)), 'lsq_data_colsum')
        return out

    def spmv_rows(self, x, first, count):
        """Rows [first, first + count) of G x (unweighted)."""
        x = as_c(x, np.float64)
        y = np.zeros(int(count))
        self._check(self._L.lsq_spmv_rows(self._h, int(first), int(count), ptr(x), ptr(y)), 'lsq_spmv_rows')
        return y


# ---- triangular kernels (drop-in signatures of the reference's Cython modules) -------------
def _tri_csr(R):
    R = sp.csr_matrix(R)
    if R.shape[0] != R.shape[1]:
        raise ValueError('R must be square')
    return (R.shape[0], as_c(R.indptr, np.int32), as_c(R.indices, np.int32), as_c(R.data, np.float64))


def _tri_check(L, rc, what):
    if rc < 0:
        raise NativeError(f'{what}: {L.tri_last_error().decode()}')
    return rc


def inv_tr_upper(R, nnz, tol, device=0):
    """LSsurf/inv_tr_upper.pyx:19 — returns (rows, cols, vals, status), same order and values."""
    L = load()
    N, rp, ci, v = _tri_csr(R)
    nnz = int(nnz)
    rr = np.zeros(nnz, np.int32)
    cc = np.zeros(nnz, np.int32)
    vv = np.zeros(nnz)
    n_out = ctypes.c_int64()
    st = _tri_check(L, L.tri_upper_inv_csr(device, N, ptr(rp), ptr(ci), ptr(v), nnz, ctypes.c_float(tol), ptr(rr),
                                           ptr(cc), ptr(vv), ctypes.byref(n_out)), 'tri_upper_inv_csr')
    k = n_out.value
    return rr[:k], cc[:k], vv[:k], st


def propagate_qz_errors(R, device=0):
    """LSsurf/propagate_qz_errors.pyx:15 — row RSS of R^-1."""
    L = load()
    N, rp, ci, v = _tri_csr(R)
    E = np.zeros(N)
    _tri_check(L, L.tri_upper_rowrss_csr(device, N, ptr(rp), ptr(ci), ptr(v), ptr(E)), 'tri_upper_rowrss_csr')
    return E


def spsolve_tr_upper(A, b, device=0):
    """LSsurf/spsolve_tr_upper.pyx:11 — x = A^-1 b for upper-triangular CSR A."""
    L = load()
    N, rp, ci, v = _tri_csr(A)
    b = as_c(b, np.float64)
    x = np.zeros(N)
    _tri_check(L, L.tri_upper_solve_csr(device, N, ptr(rp), ptr(ci), ptr(v), ptr(b), ptr(x)), 'tri_upper_solve_csr')
    return x
