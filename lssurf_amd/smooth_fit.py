"""smooth_fit — the drop-in driver, with the least-squares solve on an MI355X.

Call surface and return value follow LSsurf/smooth_fit.py:354-717 (``smooth_fit(**kwargs)``:
required data, W, ctr, spacing, E_RMS; defaults of :356-401; returns m, E, data, grids,
valid_data, TOC, R, RMS, timing, E_RMS, dzdt_lags; ``return_fit_objects`` early return of
:639-645).  What changes is underneath:

* system formation (smooth_fit.py:588-627) builds the same lin_ops on the host, but the
  weighted, column-reduced matrix ``Ip_r·TCinv·[G_data; Gc]·Ip_c`` is formed ON THE DEVICE
  once (``FitSystem``); outer iterations only re-weight and re-mask rows;
* ``sparseqr.solve`` (:142) becomes device LSQR with a warm start from the previous outer
  iteration; the residual ``G_data·m0`` (:146, :662) is a device SpMV;
* everything else (editing, sigma_extra, convergence tests, parse_model) keeps the reference's
  logic on the host.

Options that add columns/rows outside the fd_grid model (biases, sensor grids, jitter,
priors, lagrangian grids, averaging masks) are outside lssurf_amd's scope and raise
NotImplementedError instead of silently changing the fit.
"""
from time import ctime, time

import warnings
import numpy as np

from . import containers as pc
from .calc_sigma_extra import RDE, calc_sigma_extra, calc_sigma_extra_on_grid
from .constraint_functions import build_reference_epoch_matrix, node_column_blocks, \
    node_column_blocks_affine, reference_epoch_keep_cols, \
    setup_smoothness_constraints
from .grid_functions import setup_averaging_ops, setup_avg_mask_ops, setup_grids, setup_z0_avg, \
    validate_by_dz_mask
from .lin_op import known_range, lin_op, toc_range
from ._native import NativeError
from .assemble import describe
from .solver import LSQSolver

DEFAULTS = {'reference_epoch': 0, 'W_ctr': 1e4, 'return_fit_objects': False, 'mask_file': None,
            'mask_data': None, 'mask_update_function': None, 'mask_scale': {0: 10, 1: 1}, 'compute_E': False,
            'max_iterations': 10, 'min_iterations': 2, 'sigma_extra_relax': False,
            'sigma_extra_bin_spacing': None, 'sigma_extra_max': None, 'sigma_extra_keys': None,
            'srs_proj4': None, 'N_subset': None, 'bias_params': None, 'bias_filter': None, 'repeat_res': None,
            'converge_tol_dz': 0.05, 'converge_tol_frac_TSE': 0., 'DEM_tol': None, 'repeat_dt': 1,
            'Edit_only': False, 'dzdt_lags': None, 'prior_args': None, 'prior_edge_args': None,
            'avg_scales': [], 'data_slope_sensors': None, 'E_slope_bias': 0.01, 'E_RMS_d2x_PS_bias': None,
            'E_RMS_PS_bias': None, 'constraint_scaling_maps': None, 'error_res_scale': None, 'avg_masks': None,
            'sigma_extra_masks': None, 'bias_nsigma_edit': None, 'bias_nsigma_iteration': 2,
            'bias_edit_vals': None, 'sensor_grid_bias_params': None, 'ancillary_data': None,
            'lagrangian_coords': None, 'z0_average_scale': None, 'erode_source_mask': True, 'VERBOSE': True,
            'DEBUG': False,
            # lssurf_amd solver options (new keys; defaults reproduce the exact LS solution to
            # the tolerance documented in DESIGN.md §Parity)
            'device': 0, 'lsq_atol': 1e-12, 'lsq_btol': 1e-12, 'lsq_conlim': 1e12, 'lsq_maxit': 0,
            'lsq_precond': 'auto', 'lsq_dense_max': 16384, 'lsq_warm_start': True, 'lsq_method': 'auto',
            'lsq_reuse_anorm': True, 'lsq_E_method': 'auto', 'n_gpus': 1, 'devices': None}

OUT_OF_SCOPE = ('bias_params', 'sensor_grid_bias_params', 'prior_args', 'prior_edge_args', 'lagrangian_coords',
                'constraint_scaling_maps', 'mask_file', 'bias_edit_vals')


class FitSystem:
    """The device-resident smooth_fit system: G = [G_data; Gc] (unweighted COO -> device CSR),
    Ip_c as a column map; rows re-weighted / re-selected per outer iteration."""

    def __init__(self, G_data, Gc, keep_cols, n_full, device=0, structured=True, grids=None):
        self.n_data, self.n_con = int(G_data.N_eq), int(Gc.N_eq)
        self.keep_cols = keep_cols
        self.n_full = int(n_full)
        self.solver = LSQSolver(device)
        self.solver.set_col_map(self.n_full, keep_cols)
        m = self.n_data + self.n_con
        desc = describe(G_data, Gc, with_fields=True) if structured else None
        self.desc = desc           # the descriptors (bench.py's structured CPU baseline reads them)
        self.formation = 'stencil' if desc is not None else 'coo'
        if desc is not None:       # rows generated on the device from the grids and stencils
            gdesc, interp, coords, stencils, npts, fields = desc
            self.solver.set_matrix_stencil(m, self.n_full, gdesc, interp, coords, stencils, npts, fields=fields)
        else:                      # generic lin_op: host triplets -> device CSR
            r1, c1, v1 = G_data.triplets()
            r2, c2, v2 = Gc.triplets()
            self.solver.set_matrix_coo(m, self.n_full, np.concatenate([r1, r2 + self.n_data]),
                                       np.concatenate([c1, c2]), np.concatenate([v1, v2]))
        self.has_blocks = False
        self._grids, self._blocks = grids, None
        if grids is not None:      # per-node column blocks for the block-Jacobi preconditioner
            aff = node_column_blocks_affine(grids, keep_cols)
            if aff is not None:    # formed and checked on the device (no 10⁷-entry host lists)
                try:
                    self.solver.set_column_blocks_affine(*aff)
                    self.has_blocks = True
                except NativeError:
                    pass
            if not self.has_blocks:
                blocks = node_column_blocks(grids, keep_cols)
                if blocks is not None:
                    self.solver.set_column_blocks_csr(*blocks)
                    self.has_blocks = True
                    self._blocks = blocks
        self._mg = None            # multigrid (precond 4) availability, probed on first use
        self.mg_build_s = 0.0
        self.stats = None

    @property
    def blocks(self):
        """(block_ptr, cols) of the node blocks (bench.py's algorithm-matched CPU baseline), made
        on first use when the device took them in affine form."""
        if self._blocks is None and self.has_blocks:
            self._blocks = node_column_blocks(self._grids, self.keep_cols)
        return self._blocks

    def multigrid_available(self, row_weight=None):
        """True when the geometric multigrid preconditioner (lsq precond 4) runs on this system
        (structured single-GPU smooth_fit system with per-node column blocks)."""
        if self._mg is None:
            if not self.has_blocks or self.formation != 'stencil':
                self._mg = False
            else:
                if row_weight is not None and row_weight is not getattr(self, '_w_last', None):
                    self.solver.set_row_weight(row_weight)
                    self._w_last = row_weight
                tic = time()
                self._mg = bool(self.solver.cg_available(4)[0])   # builds the level hierarchy
                self.mg_build_s = time() - tic
        return self._mg

    def solve(self, row_weight, data_keep, rhs, x0=None, **opts):
        # re-upload only what changed between outer iterations (weights: same array object)
        if row_weight is not getattr(self, '_w_last', None):
            self.solver.set_row_weight(row_weight)
            self._w_last = row_weight
        dk = np.asarray(data_keep, dtype=bool)
        if getattr(self, '_keep_last', None) is None or not np.array_equal(dk, self._keep_last):
            if getattr(self, '_mask', None) is None:   # constraint rows always kept: filled once
                self._mask = np.ones(self.n_data + self.n_con, dtype=bool)
            self._mask[:self.n_data] = dk
            self.solver.set_row_mask(self._mask)
            self._keep_last = dk.copy()
        x, self.stats = self.solver.solve(rhs, x0=x0, b_rows=getattr(self, 'b_rows', 0), **opts)
        return x

    def expand(self, x):
        m0 = np.zeros(self.n_full)
        m0[self.keep_cols] = x
        return m0

    def data_forward(self, x):
        """G_data · (Ip_c x), bit-identical to scipy's csr matvec of the reference."""
        return self.solver.spmv_rows(x, 0, self.n_data)

    def rows_sumsq(self, x, ranges):
        """Per (first, count) row range of [G_data; Gc]: (Σ (w·G x)², Σ (G x)²), x compact."""
        return self.solver.rows_sumsq(x, ranges)

    def data_colsum(self, f):
        """G_dataᵀ f over the full column space (f per data row)."""
        return self.solver.data_colsum(f)

    def close(self):
        self.solver.close()


def check_data_against_DEM(in_TSE, data, m0, G_data, DEM_tol):
    m1 = m0.copy()
    m1[G_data.TOC['cols']['z0']] = 0
    r_DEM = data.z - G_data.toCSR().dot(m1) - data.DEM
    in_TSE[in_TSE] = np.abs(r_DEM[in_TSE]) < DEM_tol
    return in_TSE


def print_TOC(G_data, Gc):
    print(f'G_data : \n\t{len(np.ravel(G_data.v)) / 1000}K values\n\t shape={np.array(G_data.shape) / 1000}K')
    for label, op in (('G_data', G_data), ('Gc', Gc)):
        print(label, 'rows:')
        for name, rr in op.TOC['rows'].items():
            print(f'\t{name}: {len(np.unique(rr)) / 1000}K')


def _solve_opts(args, n, has_blocks=False, multigrid=False, dense_ok=True):
    """LSQR options.  precond 'auto': the exact dense-Cholesky preconditioner (R⁻¹ on the
    device) when n <= lsq_dense_max (one GPU only), else the geometric multigrid V-cycle
    (precond 4, CGNR) when the system supports it, else block-Jacobi per (y, x) node when the
    system has node blocks, else column scaling (maxit 50 n for the iterative ones)."""
    pc_ = args['lsq_precond']
    if pc_ == 'auto':
        pc_ = 2 if dense_ok and n <= args['lsq_dense_max'] else (4 if multigrid else (3 if has_blocks else 1))
    maxit = args['lsq_maxit'] or (0 if pc_ == 2 else 50 * n)
    # method 'auto': CGNR (normal-stencil operator, column-space only) with the iterative
    # preconditioners — the library falls back to LSQR where the structured operator is absent
    meth = {'auto': 1 if pc_ in (1, 3, 4) else 0, 'lsqr': 0, 'cgnr': 1}[args.get('lsq_method', 'auto')]
    return dict(atol=args['lsq_atol'], btol=args['lsq_btol'], conlim=args['lsq_conlim'], maxit=maxit, precond=pc_,
                method=meth)


def _anorm_seed_ok(precond, weight, in_TSE, prev):
    """May this CGNR solve seed its ‖A M^-1/2‖ estimate with the previous solve's (lsq_opts.anorm0)?
    Column scaling and node-block M: always (the preconditioned Frobenius norm is sqrt(n) whatever
    the weights and mask).  Multigrid: only with the previous solve's row weights (not after the
    sigma_extra_relax re-weighting) and at most 1 % of the data rows re-masked by the edits."""
    if precond in (1, 3):
        return True
    if prev is None or prev[0] is not weight or prev[1] is None:
        return False
    m = np.asarray(in_TSE, bool)
    return m.shape == prev[1].shape and int(np.count_nonzero(m != prev[1])) <= 0.01 * max(m.size, 1)


def iterate_fit(data, system, rhs, TCinv, G_data, Gc, in_TSE, timing, args, grids, sigma_extra_masks=None):
    """Outer editing loop (smooth_fit.py:100-210) around the device solve.  TCinv: the diagonal of
    the reference's TCinv (1/σ per row of [G_data; Gc])."""
    in_TSE_original = np.zeros(data.shape, dtype=bool)
    in_TSE_original[in_TSE] = True
    N_editable = np.sum(data.editable) if 'editable' in data.fields else data.size
    sigma_extra = np.zeros_like(data.z)
    last_iteration = args['max_iterations'] <= 1
    x = None
    rs_data = None
    timing['lsq_iters'] = 0
    # max |Δdz| between iterations (smooth_fit.py:180) on the compact solution: the dz columns are one
    # contiguous run of the ascending keep_cols, and the removed ones are 0 in every m0.  The full
    # m0 is expanded only where it is returned or read (no 10⁷-entry scatter per iteration at C4).
    dsl = _as_slice(Gc.TOC['cols']['dz'])
    kdz = tuple(int(k) for k in np.searchsorted(system.keep_cols, [dsl.start, dsl.stop])) \
        if isinstance(dsl, slice) else None
    # row weights 1/sqrt(E_all²) with E_all = 1/TCinv (smooth_fit.py:103, 129): |TCinv| — the caller's
    # array itself when positive (no pass over, or copy of, the 77 M rows at C4).  sqrt(fl(x²)) = |x|
    # in IEEE arithmetic, so the reference's weight is 1/|fl(1/TCinv)|, which can differ from |TCinv|
    # by one ulp (a relative 1e-16 change of a row weight; DESIGN.md §4 records the deviation).  The
    # weights are a read-only view: nothing may edit them in place, since they alias TCinv.
    weight0 = (TCinv if TCinv.min() > 0 else np.abs(TCinv)).view()
    weight0.flags.writeable = False
    prev_solve = None   # (row weights, data-row mask) of the previous solve: _anorm_seed_ok
    for iteration in range(args['max_iterations']):
        weight = weight0
        if last_iteration and args['sigma_extra_relax']:
            if args['VERBOSE']:
                print('smooth_fit.iterate_fit: relaxing errors by sigma_extra')
            nd = G_data.shape[0]   # E2_plus = E_all² + sigma_extra² on the data rows only
            weight = weight0.copy()
            weight[:nd] = 1. / np.sqrt((1. / TCinv[:nd]) ** 2 + sigma_extra ** 2)
        if args['VERBOSE']:
            print('starting device lsqr solve for iteration %d at %s' % (iteration, ctime()), flush=True)
        tic = time()
        x_last = x
        x0 = x if (args['lsq_warm_start'] and x is not None) else None
        dense_ok = getattr(system, 'dense_ok', True)
        mg = args['lsq_precond'] == 'auto' and (system.keep_cols.size > args['lsq_dense_max'] or not dense_ok) and \
            system.multigrid_available(weight)
        if mg and 'mg_build' not in timing:
            timing['mg_build'] = system.mg_build_s
        opts = _solve_opts(args, system.keep_cols.size, system.has_blocks, mg, dense_ok)
        last = system.stats
        if args['lsq_reuse_anorm'] and last is not None and last.get('method') == 1 and \
                opts['method'] == 1 and last.get('precond') == opts['precond'] and \
                _anorm_seed_ok(opts['precond'], weight, in_TSE, prev_solve):
            # the CGNR stopping rule starts from the previous solve's ‖A M^-1/2‖ estimate (lsq_opts
            # .anorm0) instead of rebuilding it from zero: with node-block M (or column scaling) the
            # preconditioned Frobenius norm is sqrt(n) whatever the weights, so the estimate stays
            # below it.  The multigrid M has no such invariant: there the seed is taken only when
            # the weights are the previous solve's and at most 1 % of the data rows changed mask
            opts['anorm0'] = float(last['anorm'])
        try:
            x = system.solve(weight, in_TSE, rhs, x0=x0, **opts)
        except NativeError as e:
            if opts['precond'] != 4:
                raise
            # the multigrid set-up can fail for these weights (e.g. a coarsest level that is not
            # positive definite): the block-Jacobi solve still reaches the same solution
            print(f'smooth_fit: multigrid preconditioner unavailable ({e}); block-Jacobi for the rest of '
                  f'the fit', flush=True)
            system._mg = False
            opts = _solve_opts(args, system.keep_cols.size, system.has_blocks, False, dense_ok)
            x = system.solve(weight, in_TSE, rhs, x0=x0, **opts)
        if system.stats['istop'] == 7:
            print(f"smooth_fit: LSQR reached its iteration limit ({system.stats['iters']}) before the "
                  f"requested tolerance; raise lsq_maxit or use lsq_precond=2", flush=True)
        system.stats['precond'] = opts['precond']
        prev_solve = (weight, np.asarray(in_TSE, bool).copy() if opts['precond'] == 4 else None)
        system.last_x = x   # compact solution: z_est and the constraint statistics read it, not m0
        timing['sparseqr_solve'] = time() - tic
        timing['lsq_iters'] += int(system.stats['iters'])
        timing.setdefault('lsq_iters_per_solve', []).append(int(system.stats['iters']))
        timing['lsq_setup'] = timing.get('lsq_setup', 0.) + float(system.stats.get('setup_s', 0.))
        timing['lsq_last'] = dict(system.stats)
        tic = time()
        r_data = data.z - system.data_forward(x)
        rs_data = r_data / data.sigma
        timing['residual'] = timing.get('residual', 0.) + time() - tic
        if last_iteration:
            break
        tic_edit = time()
        if args.get('sigma_extra_bin_spacing') is None:
            sigma_extra = calc_sigma_extra(r_data, data.sigma, in_TSE, sigma_extra_masks, device=args['device'])
        else:
            sigma_extra = calc_sigma_extra_on_grid(data.x, data.y, r_data, data.sigma, in_TSE,
                                                   sigma_extra_masks=sigma_extra_masks,
                                                   sigma_extra_max=args['sigma_extra_max'],
                                                   spacing=args['sigma_extra_bin_spacing'])
        sigma_aug = np.sqrt(data.sigma ** 2 + sigma_extra ** 2)
        in_TSE_last = in_TSE
        in_TSE = np.abs(r_data / sigma_aug) < 3.0
        bias_editing_changed = False
        if 'editable' in data.fields:
            in_TSE[data.editable == 0] = in_TSE_original[data.editable == 0]
        if args['DEM_tol'] is not None:
            in_TSE = check_data_against_DEM(in_TSE, data, system.expand(x), G_data, args['DEM_tol'])
        if not np.any(in_TSE):
            if args['VERBOSE']:
                print('Edited data empty, returning')
            return system.expand(x), sigma_extra, in_TSE, rs_data
        if kdz is not None:
            xs = x[kdz[0]:kdz[1]]
            ddz = np.abs(xs) if x_last is None else np.subtract(x_last[kdz[0]:kdz[1]], xs)
            dmax = float(np.max(np.abs(ddz, out=ddz))) if ddz.size else 0.0
        else:
            m_last = system.expand(x_last) if x_last is not None else np.zeros(system.n_full)
            dmax = float(np.max(np.abs(m_last[dsl] - system.expand(x)[dsl])))
        if dmax < args['converge_tol_dz'] and iteration > args['min_iterations']:
            if args['VERBOSE']:
                print('Solution identical to previous iteration with tolerance %3.1f, exiting after iteration %d'
                      % (args['converge_tol_dz'], iteration))
            last_iteration = True
        if args['VERBOSE']:
            print('found %d in TSE, dt=%3.0f' % (in_TSE.sum(), timing['sparseqr_solve']), flush=True)
            if sigma_extra_masks is None:
                print(f'\t median(sigma_extra)={np.median(sigma_extra):3.4f}')
            else:
                for key, ii in sigma_extra_masks.items():
                    print(f'\t sigma_extra for {key} : {np.median(sigma_extra[ii]):3.4f}', flush=True)
                for key, ii in sigma_extra_masks.items():
                    print(f'\t sigma_hat for {key} : {RDE(r_data[ii] / sigma_aug[ii]):3.4f}', flush=True)
        if iteration > 0 and iteration > args['bias_nsigma_iteration']:
            frac_TSE_change = len(np.setxor1d(in_TSE_last, in_TSE)) / N_editable
            if frac_TSE_change < args['converge_tol_frac_TSE']:
                if args['VERBOSE']:
                    print('filtering unchanged with tolerance %3.5f, will exit after iteration %d'
                          % (args['converge_tol_frac_TSE'], iteration + 1))
                last_iteration = True
        if iteration >= np.maximum(args['min_iterations'], args['bias_nsigma_iteration'] + 1):
            if np.all(sigma_extra < 0.5 * np.min(data.sigma[in_TSE])) and not bias_editing_changed:
                if args['VERBOSE']:
                    print('sigma_extra is small, performing one additional iteration', flush=True)
                last_iteration = True
        if iteration == args['max_iterations'] - 2:
            last_iteration = True
        timing['edit'] = timing.get('edit', 0.) + time() - tic_edit
    return (system.expand(x) if x is not None else np.zeros(system.n_full)), sigma_extra, in_TSE, rs_data


def _toc_slice(op, name):
    """op.TOC['rows'][name] as a slice when it is one contiguous run (not materialised), else the
    index array"""
    kr = toc_range(op.TOC['rows'], name)
    return slice(kr[0], kr[1] + 1) if kr is not None else _as_slice(op.TOC['rows'][name])


def _as_slice(idx):
    """A contiguous ascending index array as a slice (no fancy-indexing copy of 73 M rows)."""
    kr = known_range(idx)
    if kr is not None:
        return slice(kr[0], kr[1] + 1)
    idx = np.asarray(idx)
    if idx.ndim == 1 and idx.size and idx[-1] - idx[0] == idx.size - 1 and np.all(idx[1:] - idx[:-1] == 1):
        return slice(int(idx[0]), int(idx[-1]) + 1)
    return idx


def _device_constraint_stats(system, m0, Gc, R, RMS):
    """R and RMS of each constraint type (smooth_fit.py:318-331) reduced on the device from the
    formed operator: no host copy of the 10⁷–10⁸ constraint residuals.  False when a type's rows
    are not one contiguous range (then the caller takes the host path)."""
    names, ranges = [], []
    for eq_type in ['d2z_dt2', 'grad2_z0', 'grad2_dzdt', 'grad2_PS']:
        if eq_type in Gc.TOC['rows']:
            rows = _toc_slice(Gc, eq_type)
            if not isinstance(rows, slice):
                return False
            names.append(eq_type)
            ranges.append((system.n_data + rows.start, rows.stop - rows.start))
    if names:
        x = getattr(system, 'last_x', None)   # the compact solution m0 was expanded from (iterate_fit)
        if x is None or x.size != np.size(system.keep_cols):
            x = m0[system.keep_cols]
        sw, su = system.rows_sumsq(x, ranges)
        for name, (first, count), a, b in zip(names, ranges, sw, su):
            R[name] = a
            RMS[name] = np.sqrt(b / count)
    return True


def tcinv_diagonal(Ed, Gc, constraint_op_list):
    """The diagonal of TCinv = diag(1 / [Ed; Ec]) (smooth_fit.py:594-613), written in one pass from
    the ops' expected values (no Ec, no concatenation of the 77 M rows at C4); equal bit for bit to
    1 / np.concatenate((Ed, Ec)).  A constraint row that no op covers has Ec = 0 there: the
    reference's zero check (the ops' own expected values were checked by
    setup_smoothness_constraints)."""
    nd = Ed.size
    out = np.empty(nd + Gc.N_eq)
    np.divide(1., Ed, out=out[:nd])
    Tc = out[nd:]
    covered = 0
    for op in constraint_op_list:
        rows = _toc_slice(Gc, op.name)
        e = np.ravel(op.expected)
        if isinstance(rows, slice):
            np.divide(1., e, out=Tc[rows])
            covered += rows.stop - rows.start
        else:
            Tc[rows] = 1. / e
            covered += np.size(rows)
    if covered != Gc.N_eq:
        raise ValueError('zero value found in constraint sigma')
    return out


def parse_model(m, m0, data, R, RMS, G_data, averaging_ops, Gc, Ec, grids, args, ru=None, system=None):
    """Output grids and fit statistics (smooth_fit.py:276-352).  With the device `system` the
    constraint statistics and the count / misfit maps are reduced on the device."""
    z0g, dzg = grids['z0'], grids['dz']
    # the column ranges as slices (a copy of a slice, not a 12 M-entry gather at C4)
    cols_of = {ff: _as_slice(G_data.TOC['cols'][ff]) for ff in ('z0', 'dz')}
    m['z0'] = pc.grid.data().from_dict({'x': z0g.ctrs[1], 'y': z0g.ctrs[0], 'cell_area': z0g.cell_area,
                                        'mask': z0g.mask, 'z0': np.reshape(np.array(m0[cols_of['z0']]), z0g.shape)})
    m['dz'] = pc.grid.data().from_dict({'x': dzg.ctrs[1], 'y': dzg.ctrs[0], 'time': dzg.ctrs[2],
                                        'dz': np.reshape(np.array(m0[cols_of['dz']]), dzg.shape),
                                        'cell_area': dzg.cell_area, 'mask': dzg.mask})
    for key, op in averaging_ops.items():
        fields = {coord: ctr for coord, ctr in zip(op.dst_grid.coords, op.dst_grid.ctrs)}
        fields.update({'cell_area': op.dst_grid.cell_area, key: op.grid_prod(m0)})
        m[key] = pc.grid.data().from_dict(fields)
    m['all'] = m0
    m['extent'] = np.concatenate((z0g.bds[1], z0g.bds[0]))
    m['sensor_bias_grids'] = {}
    m['jitter_bias_grids'] = {}
    if system is None or not _device_constraint_stats(system, m0, Gc, R, RMS):
        if callable(Ec):         # smooth_fit's on-demand constraint sigma
            Ec = Ec()
        if ru is None:           # unscaled constraint residuals Gc·m0 (device product when available)
            ru = system.solver.spmv(m0[system.keep_cols])[system.n_data:] if hasattr(system, 'solver') \
                else Gc.toCSR().dot(m0)
        for eq_type in ['d2z_dt2', 'grad2_z0', 'grad2_dzdt', 'grad2_PS']:
            if eq_type in Gc.TOC['rows']:
                rows = _toc_slice(Gc, eq_type)
                rc = (1. / Ec[rows]) * ru[rows]   # TCinv_cov.dot(ru), smooth_fit.py:324-326
                R[eq_type] = np.sum(rc ** 2)
                RMS[eq_type] = np.sqrt(np.mean(ru[rows] ** 2))
    tse = data.three_sigma_edit
    r = (data.z - data.z_est)[tse]
    if args['sigma_extra_relax']:
        r_scaled = r / np.sqrt(data.sigma[tse] ** 2 + data.sigma_extra[tse] ** 2)
    else:
        r_scaled = r / data.sigma[tse]
    # Gselᵀ·{1, r_scaled², r²} of smooth_fit.py:341-347: weighted column sums over the kept data rows
    per_point = {'scaled': r_scaled ** 2, 'plain': r ** 2}
    if 'tide' in data.fields:   # smooth_fit.py:346-352: the residual with the tide correction undone
        r_notide = (data.z + data.tide - data.z_est)[tse]
        per_point['notide_plain'] = r_notide ** 2
        per_point['notide_scaled'] = (r_notide / data.sigma[tse]) ** 2
    tse_b = np.asarray(tse).astype(bool).ravel()
    n_cols = G_data.col_N
    sums = None
    if system is not None and getattr(system, 'formation', None) == 'stencil':
        fs = {'count': tse_b.astype(float)}
        for key, vals in per_point.items():
            f = np.zeros(tse_b.size)
            f[tse_b] = vals
            fs[key] = f
        try:   # node gather over the points sorted by cell (no host triplets of the data operator)
            sums = {k: system.data_colsum(f)[:n_cols] for k, f in fs.items()}
        except NativeError:
            sums = None
    if sums is None:   # host: weighted column sums of G_data's triplets
        rr, cc, vv = G_data.triplets()
        rows_tse = np.flatnonzero(tse_b)
        pos = np.full(tse_b.shape, -1)
        pos[rows_tse] = np.arange(rows_tse.size)
        sel = tse_b[rr] & (vv != 0)
        c_sel, v_sel, p_sel = cc[sel], vv[sel], pos[rr[sel]]
        sums = {'count': np.bincount(c_sel, weights=v_sel, minlength=n_cols)}
        for key, vals in per_point.items():
            sums[key] = np.bincount(c_sel, weights=v_sel * vals[p_sel], minlength=n_cols)
    for ff in ['dz', 'z0']:
        cols = cols_of[ff]
        shape = grids[ff].shape
        m[ff].assign({'count': sums['count'][cols].reshape(shape)})
        m[ff].count[m[ff].count == 0] = np.nan
        m[ff].assign({'misfit_scaled_rms': np.sqrt(sums['scaled'][cols].reshape(shape) / m[ff].count)})
        m[ff].assign({'misfit_rms': np.sqrt(sums['plain'][cols].reshape(shape) / m[ff].count)})
        if 'notide_plain' in sums:
            m[ff].assign({'misfit_notide_rms': np.sqrt(sums['notide_plain'][cols].reshape(shape) / m[ff].count)})
            m[ff].assign({'misfit_notide_scaled_rms':
                          np.sqrt(sums['notide_scaled'][cols].reshape(shape) / m[ff].count)})


def smooth_fit(**kwargs):
    required = ('data', 'W', 'ctr', 'spacing', 'E_RMS')
    args = dict(DEFAULTS)
    args.update(kwargs)
    for field in required:
        if field not in kwargs:
            raise ValueError('%s must be defined' % field)
    for key in OUT_OF_SCOPE:
        if args.get(key) is not None:
            raise NotImplementedError(f'smooth_fit: {key!r} is outside lssurf_amd (SURVEY.md §2)')
    if args.get('data_slope_sensors') is not None and len(args['data_slope_sensors']) > 0:
        raise NotImplementedError("smooth_fit: 'data_slope_sensors' is outside lssurf_amd")

    valid_data = np.isfinite(args['data'].z)
    if 'sensor' not in args['data'].fields:
        args['data'].assign(sensor=np.zeros(args['data'].shape))
    timing = {}
    m, E, R, RMS = {}, {}, {}, {}
    tic = time()
    grids, bds = setup_grids(args)
    valid_data = valid_data & grids['dz'].validate_pts(args['data'].coords()) & \
        grids['z0'].validate_pts(args['data'].coords()[0:2])
    if not np.any(valid_data):
        if args['VERBOSE']:
            print('smooth_fit: no valid data')
        return {'m': m, 'E': E, 'data': None, 'grids': grids, 'valid_data': valid_data, 'TOC': {}, 'R': {},
                'RMS': {}, 'timing': timing, 'E_RMS': args['E_RMS']}
    data = args['data'].copy_subset(valid_data)
    validate_by_dz_mask(data, grids, valid_data)
    if args['sigma_extra_keys'] is not None:
        # one sigma_extra group per key: the data whose field takes any of the listed values
        # (smooth_fit.py:442-447; the masks are over the valid subset already)
        args['sigma_extra_masks'] = {}
        for key, field_vals in args['sigma_extra_keys'].items():
            mask = np.zeros_like(data.sensor, dtype=bool)
            for field, vals in field_vals.items():
                mask |= np.isin(getattr(data, field), vals)
            args['sigma_extra_masks'][key] = mask
    elif args['sigma_extra_masks'] is not None:
        for key in args['sigma_extra_masks']:
            args['sigma_extra_masks'][key] = args['sigma_extra_masks'][key][valid_data == 1]
    if data.size == 0:
        print('\tsmooth_fit.py: after masking, no data found')
        return {'m': m, 'E': E, 'data': data, 'grids': grids, 'valid_data': valid_data, 'TOC': {}, 'R': {},
                'RMS': {}, 'timing': timing, 'E_RMS': args['E_RMS']}

    G_data = lin_op(grids['z0'], name='interp_z').interp_mtx(data.coords()[0:2])
    G_data.add(lin_op(grids['dz'], name='interp_dz').interp_mtx(data.coords()))
    constraint_op_list = []
    if args['VERBOSE']:
        print(f"smooth_fit: E_RMS={args['E_RMS']}")
    setup_smoothness_constraints(grids, constraint_op_list, args['E_RMS'], args['mask_scale'])
    zero_prior = set()   # priors created here are zeros: rhs is already zero on their rows
    for op in constraint_op_list:
        if op.prior is None:
            op.prior = np.zeros(np.shape(op.expected))   # calloc: untouched pages (73 M rows at C4)
            zero_prior.add(op.name)
    Gc = lin_op(None, name='constraints').vstack(constraint_op_list)
    N_eq = G_data.N_eq + Gc.N_eq
    Ed = data.sigma.ravel()
    if not np.all(Ed):     # no boolean temporary
        raise ValueError('zero value found in data sigma')
    TCinv_diag = tcinv_diagonal(Ed, Gc, constraint_op_list)

    def Ec():   # the reference reads Ec only as 1/Ec: made on demand (73 M rows at C4)
        out = np.zeros(Gc.N_eq)
        for op in constraint_op_list:
            out[_toc_slice(Gc, op.name)] = op.expected
        return out
    if args['DEBUG']:
        print_TOC(G_data, Gc)
    rhs = np.zeros([N_eq])
    rhs[0:data.size] = data.z.ravel()
    b_rows = data.size   # rhs[b_rows:] == 0: only the data rows (and non-zero priors) cross PCIe
    for op in constraint_op_list:   # rhs[data.size:] = the concatenated priors
        if op.name not in zero_prior:
            rows = _toc_slice(Gc, op.name)
            prior = np.ravel(op.prior)
            if isinstance(rows, slice):
                rhs[data.size + rows.start:data.size + rows.stop] = prior
                end = rows.stop
            else:
                rhs[data.size + rows] = prior
                end = int(np.max(rows)) + 1 if np.size(rows) else 0
            if np.any(prior != 0):
                b_rows = max(b_rows, data.size + end)
    keep_cols = reference_epoch_keep_cols(G_data.col_N, grids['dz'], args['reference_epoch'])
    timing['setup'] = time() - tic
    in_TSE = data.three_sigma_edit > 0.01 if 'three_sigma_edit' in data.fields else np.ones(G_data.N_eq, dtype=bool)
    if args['VERBOSE']:
        print('initial: %d:' % np.max(G_data.r), flush=True)
    if args['return_fit_objects']:
        return {'data': data, 'G_data': G_data, 'Gc': Gc, 'grids': grids, 'Ed': Ed, 'Ec': Ec()}

    system = None
    try:
        if args['max_iterations'] > 0:
            tic = time()
            devices = args['devices'] if args['devices'] is not None else \
                [args['device'] + k for k in range(int(args['n_gpus']))]
            if len(devices) > 1:   # y-slab ranks on several devices of this process (lssurf_amd.dist)
                from .dist import MultiDeviceFitSystem
                if len(set(devices)) > 1:
                    warnings.warn('smooth_fit(n_gpus > 1) on distinct devices: the threaded device-group '
                                  'path (one RCCL communicator per device) has been tested only as ranks '
                                  'sharing one device; see INTEGRATION.md §5', RuntimeWarning, stacklevel=2)
                system = MultiDeviceFitSystem(G_data, Gc, keep_cols, Gc.col_N, devices)
            else:
                system = FitSystem(G_data, Gc, keep_cols, Gc.col_N, device=devices[0], grids=grids)
            system.b_rows = b_rows
            timing['device_setup'] = time() - tic
            tic_iteration = time()
            m0, sigma_extra, in_TSE, rs_data = iterate_fit(data, system, rhs, TCinv_diag, G_data, Gc, in_TSE,
                                                           timing, args, grids,
                                                           sigma_extra_masks=args['sigma_extra_masks'])
            timing['iteration'] = time() - tic_iteration
            valid_data[valid_data] = in_TSE
            data.assign({'three_sigma_edit': in_TSE})
            data.assign({'sigma_extra': sigma_extra})
            x_c = getattr(system, 'last_x', None)   # m0[keep_cols], without the 10⁷-entry gather
            data.assign({'z_est': np.reshape(system.data_forward(x_c if x_c is not None else m0[keep_cols]),
                                             data.shape)})
            if args['mask_update_function'] is not None:
                averaging_ops = {}
                parse_model(m, m0, data, R, RMS, G_data, averaging_ops, Gc, Ec(), grids, args)
                args['mask_update_function'](grids, m, args)
            averaging_ops = setup_averaging_ops(grids['dz'], grids['dz'].col_N, args, grids['dz'].cell_area)
            averaging_ops.update(setup_z0_avg(grids, grids['dz'].col_N, args))
            averaging_ops.update(setup_avg_mask_ops(grids['dz'], G_data.col_N, args['avg_masks'], args['dzdt_lags']))
            parse_model(m, m0, data, R, RMS, G_data, averaging_ops, Gc, Ec, grids, args, system=system)
            tse = data.three_sigma_edit == 1
            r_data = data.z_est[tse] - data.z[tse]
            R['data'] = np.sum((r_data / data.sigma[tse]) ** 2)
            RMS['data'] = np.sqrt(np.mean(r_data ** 2))
        else:
            averaging_ops = setup_averaging_ops(grids['dz'], grids['dz'].col_N, args, grids['dz'].cell_area)
            averaging_ops.update(setup_z0_avg(grids, grids['dz'].col_N, args))
            averaging_ops.update(setup_avg_mask_ops(grids['dz'], G_data.col_N, args['avg_masks'], args['dzdt_lags']))
        if args['compute_E']:
            from .errors import calc_and_parse_errors
            if 'sigma_extra' not in data.fields:
                data.assign({'sigma_extra': np.zeros_like(data.sigma)})
                tse = data.three_sigma_edit == 1
                r_data = data.z_est[tse] - data.z[tse]
                data.sigma_extra[tse] = calc_sigma_extra(r_data, data.sigma[tse], np.ones(tse.sum(), dtype=bool))
            if args['VERBOSE']:
                print('Starting uncertainty calculation', flush=True)
                tic_error = time()
            calc_and_parse_errors(E, G_data, Gc, Ed, Ec(), data, in_TSE, keep_cols, grids, averaging_ops,
                                  device=args['device'], timing=timing, method=args['lsq_E_method'])
            if args['VERBOSE']:
                print('\tUncertainty propagation took %3.2f seconds' % (time() - tic_error), flush=True)
    finally:
        if system is not None:
            system.close()
    return {'m': m, 'E': E, 'data': data, 'grids': grids, 'valid_data': valid_data, 'TOC': Gc.TOC, 'R': R,
            'RMS': RMS, 'timing': timing, 'E_RMS': args['E_RMS'], 'dzdt_lags': args['dzdt_lags']}


# re-exported for callers that build Ip_c explicitly (smooth_fit.py:624)
__all__ = ['smooth_fit', 'iterate_fit', 'parse_model', 'FitSystem', 'build_reference_epoch_matrix',
           'check_data_against_DEM']
