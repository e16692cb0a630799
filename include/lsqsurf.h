/*
 * lsqsurf.h — C ABI of lssurf_amd's MI355X (gfx950) least-squares solve path.
 *
 * This is the only public native surface (liblsqsurf.so).  It replaces, for LSsurf's
 * sparse regularized least-squares solve path:
 *
 *   sparseqr.solve(A, b)               LSsurf/smooth_fit.py:142 (iterate_fit),
 *                                      notebooks/smooth_fit_demo_aniso.ipynb cells 6,13,16,18,20
 *       -> lsq_create / lsq_set_col_map / lsq_set_matrix_coo / lsq_set_row_weight /
 *          lsq_set_row_mask / lsq_solve
 *   G_data.toCSR().dot(m0)             LSsurf/smooth_fit.py:146,662 (residual / z_est)
 *       -> lsq_spmv
 *   Gcoo = sp.vstack([...]).tocoo()·Ip_c, TCinv·Gcoo, Ip_r·(...)   smooth_fit.py:613-627,123-142
 *       -> formed on the device by lsq_set_matrix_coo (+col map, row weight, row mask)
 *   inv_tr_upper(R, nnz, tol)          LSsurf/inv_tr_upper.pyx:19-94 (smooth_fit.py:240-246)
 *       -> tri_upper_inv_csr
 *   propagate_qz_errors(R)             LSsurf/propagate_qz_errors.pyx:15-69
 *       -> tri_upper_rowrss_csr
 *   spsolve_tr_upper(A, b)             LSsurf/spsolve_tr_upper.pyx:11-54
 *       -> tri_upper_solve_csr
 *
 * Conventions
 *   - Ownership: the caller owns every host buffer; the library copies in and out and owns all
 *     device memory.  Pointers are plain host pointers, sizes are int64.
 *   - Errors: int return, 0 = ok, 1 = "not converged" (lsq_solve hit maxit) or "output buffer
 *     full" (tri_upper_inv_csr, same meaning as inv_tr_upper's status=1); < 0 = invalid
 *     argument / call order / HIP error, with lsq_last_error() describing it; -5 = declined for
 *     lack of resources (a band factor that does not fit the device or exceeds the width limit —
 *     the caller may choose another preconditioner).  There is no CPU fallback: without a
 *     usable gfx950 device every call fails.
 *   - Threading: one handle per host thread; calls on one handle are serialised.
 */
#ifndef LSQSURF_H
#define LSQSURF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lsq_handle lsq_handle;

/* Solver options.  Defaults (lsq_default_opts) reproduce scipy.sparse.linalg.lsqr's stopping
 * rules with atol = btol = 1e-10, conlim = 1e8, maxit = 4*n. */
typedef struct lsq_opts {
    int32_t method;        /* 0 = LSQR (Paige & Saunders 1982); 1 = CGNR: preconditioned CG on  */
                           /*     the normal equations with the fused normal-stencil operator   */
                           /*     (structured systems, single-GPU or structured ranks; precond  */
                           /*     1, 3 or 4; other single-GPU systems fall back to LSQR and     */
                           /*     report method 0 in lsq_stats)                                 */
    int32_t precond;       /* 0 = none, 1 = column (Jacobi) scaling, 2 = dense Cholesky R⁻¹   */
                           /*     (exact right preconditioner; n up to a few 10^4), 3 = block-  */
                           /*     Jacobi: R_b⁻¹ of every column block (lsq_set_column_blocks;   */
                           /*     SURVEY.md §8 a7.4 — no reference counterpart), 4 = geometric  */
                           /*     multigrid V-cycle over the (y, x) node lattice (method 1,     */
                           /*     smooth_fit systems with per-node column blocks, single GPU or */
                           /*     structured ranks with lsq_dist_set_global; DESIGN.md          */
                           /*     §Multigrid), 5 = banded Cholesky R̃⁻¹ in the order of         */
                           /*     lsq_set_band_order (LSQR, single GPU; band.hip)               */
    double  atol, btol, conlim;
    int64_t maxit;
    int32_t use_x0;        /* 1: x_inout holds a warm start (outer-iteration "resume")          */
    int32_t batch;         /* iterations per device batch between host convergence checks      */
    int32_t use_graph;     /* 1: replay each batch as a captured hipGraph                       */
    int32_t op;            /* operator the iteration streams: 0 = auto (the structured stencil  */
                           /*     operator when the matrix came from lsq_set_matrix_stencil and */
                           /*     precond < 2; else assembled SELL), 1 = assembled SELL always  */
    int64_t b_rows;        /* rows of b that may be non-zero: b[0, b_rows) is uploaded, the     */
                           /*     rest taken as zero (smooth_fit: the data rows, when no prior  */
                           /*     is non-zero); 0 = all m rows                                 */
    double  anorm0;        /* CGNR: an ‖A‖ estimate to start the stopping rule from — lsq_stats */
                           /*     .anorm of an earlier solve of the same operator and           */
                           /*     preconditioner (smooth_fit's later outer solves, warm         */
                           /*     starts).  The rule uses max(anorm0, the running Lanczos       */
                           /*     estimate), which only grows towards the true norm; without it */
                           /*     a re-solve from the solution iterates until the estimate has  */
                           /*     rebuilt.  0 = none (scipy's rule); ignored by LSQR            */
} lsq_opts;

/* Statistics (mirrors scipy's lsqr return tuple, plus timing and the byte model). */
typedef struct lsq_stats {
    int64_t iters;
    int32_t istop;         /* scipy istop: 1,2 converged; 3 cond limit; 4-6 machine precision; 7 maxit */
    int32_t method;        /* method that ran: 0 LSQR, 1 CGNR (acond is not estimated: 0)      */
    double  r1norm, r2norm, anorm, acond, arnorm, xnorm;
    double  time_s;        /* device-resident iteration time (A, b already in HBM)              */
    double  bytes_per_iter;/* algorithmic HBM bytes of one LSQR iteration (DESIGN.md byte model)*/
    double  setup_s;       /* CGNR: per-solve preconditioner set-up and initialisation (block   */
                           /*     factors, multigrid levels and λ estimates), host wall clock, */
                           /*     not part of time_s; LSQR: 0                                  */
    double  comm_bytes_per_iter; /* distributed CGNR: bytes one rank sends per iteration (halos   */
                           /*     and all-reduces; the busiest rank of a virtual / device group); */
                           /*     0 on one GPU                                                  */
} lsq_stats;

void        lsq_default_opts(lsq_opts* o);

/* ---- handle lifetime -------------------------------------------------------------------- */
lsq_handle* lsq_create(int32_t device);
void        lsq_destroy(lsq_handle* h);
const char* lsq_last_error(lsq_handle* h);     /* never NULL; "" when no error                 */

/* ---- matrix formation (replaces the scipy assembly of smooth_fit.py:613-627) ------------ */
/* Optional, before lsq_set_matrix_coo: keep only these columns of the full operator, in this
 * order (= Ip_c of build_reference_epoch_matrix, constraint_functions.py:112-151). keep_cols
 * must be strictly increasing in [0, n). */
int lsq_set_col_map(lsq_handle* h, int64_t n_full, const int64_t* keep_cols, int64_t n_keep);

/* Form A = diag(row_weight) * G * Ip_c on the device from COO triplets of G (m x n_full):
 * entries with v == 0 are dropped, duplicates are summed in input order, sums equal to 0 are
 * dropped, columns outside the col map are removed (lin_op.toCSR, lin_op.py:745-753, plus the
 * scipy products of smooth_fit.py:613-627).  row_weight may be NULL (= 1).  Builds A and Aᵀ. */
int lsq_set_matrix_coo(lsq_handle* h, int64_t m, int64_t n_full, int64_t nnz,
                       const int64_t* r, const int64_t* c, const double* v,
                       const double* row_weight);

/* Structured formation (no host triplets): the smooth_fit operator described by its fd_grids
 * and stencils, rows generated on the device exactly as lin_op would generate them.
 *   data rows 0..npts-1: sum over `n_interp` interpolation parts (lin_op.interp_mtx,
 *     lin_op.py:163-247) of point p = (py, px[, pt]) on grid interp_grid[k]; points must be
 *     inside every grid (bounds_error=True semantics);
 *   stencil part s covers rows [row0, row0+n_eq): centre k -> subscripts lo + unravel(k, hi-lo)
 *     ('ij' meshgrid order), entries col0 + ravel(centre + off[t]) with value val[t]
 *     (lin_op.diff_op, lin_op.py:80-132).
 * Then the same zero-drop / duplicate-sum / col-map rules as lsq_set_matrix_coo. */
typedef struct lsq_grid_desc {
    int32_t ndim, reserved;
    int64_t shape[3];
    int64_t col0;
    double  b0[3], delta[3];
} lsq_grid_desc;
typedef struct lsq_stencil_desc {
    int32_t grid, ntpl;
    int32_t off[8][3];
    double  val[8];
    int64_t row0, n_eq;
    int64_t lo[3], hi[3];
} lsq_stencil_desc;
int lsq_set_matrix_stencil(lsq_handle* h, int64_t m, int64_t n_full,
                           int32_t n_grids, const lsq_grid_desc* grids,
                           int32_t n_interp, const int32_t* interp_grid, int64_t npts,
                           const double* py, const double* px, const double* pt,
                           int32_t n_stencil, const lsq_stencil_desc* stencils,
                           const double* row_weight);

/* Field-valued (variable-coefficient) stencil part, staged before lsq_set_matrix_stencil: stencil
 * index `stencil` of that call keeps its grid, rows and centre box, and its template becomes the
 * ntpl (≤ 16) offsets off[3·t + d] with entry value val[t] · F[fsel[t]·n_eq + k] in the row of
 * centre k (k = ravel of centre − lo over the box, the row order of lin_op.diff_op).  F holds the
 * nfield exact per-row values (field-major).  This is the directional smoothing operator of
 * notebooks/smooth_fit_demo_aniso.ipynb cells 9-10: a lin_op.diff_op template whose rows
 * scale_op_by_2d_grid multiplies by the interpolated direction field (u², 2uv, v²), summed over
 * three templates on the same rows — one part here, 9 entries, F = the distinct |values|. */
int lsq_set_stencil_fields(lsq_handle* h, int32_t stencil, int32_t ntpl, const int32_t* off, const double* val,
                           int32_t nfield, const int32_t* fsel, int64_t n_eq, const double* F);

/* Replace the row weights (TCinv of iterate_fit, smooth_fit.py:123-129) without re-forming. */
int lsq_set_row_weight(lsq_handle* h, const double* row_weight);
/* Row selection Ip_r (smooth_fit.py:132-135): rows with keep[i] == 0 are excluded from the
 * fit (treated as absent rows).  NULL keeps every row. */
int lsq_set_row_mask(lsq_handle* h, const uint8_t* keep);
/* Column blocks of the block-Jacobi preconditioner (precond 3): block b holds the compact
 * columns cols[block_ptr[b] .. block_ptr[b+1]) (at most 16, each column in at most one block);
 * unlisted columns are singleton blocks.  For smooth_fit a block is one (y, x) node: its z0
 * column and its dz columns of every kept epoch.  The factors R_b (AᵀA restricted to the block
 * = R_bᵀR_b, with the current row weights / mask) are rebuilt on the device when weights change;
 * R_b⁻¹ is kept rounded to bf16 (products in f64), the same M for CGNR and for every use LSQR
 * makes of it, so x is unaffected (any non-singular M gives the same least-squares solution).
 * NULL / 0 blocks clears the structure (every column its own block).  On a structured rank
 * (lsq_dist_set_halo) the blocks are the rank's owned nodes in its local compact ids, factored
 * from the rank's own rows; ghost columns stay outside every block. */
int lsq_set_column_blocks(lsq_handle* h, int64_t n_blocks, const int64_t* block_ptr, const int32_t* cols);
/* The same blocks given by their affine structure, as smooth_fit's node blocks are (single-GPU
 * handles): block b (0 <= b < n_blocks) holds the k <= 16 compact columns base[j] + b*stride[j],
 * whose full columns (lsq_set_col_map) are full_base[j] + b*full_stride[j].  The blocks must cover
 * every compact column exactly once (n_blocks*k == n).  The library forms the block arrays on the
 * device and checks all of this there (no 10^7-entry host column lists); on a violation it
 * returns < 0 and leaves no blocks set.  Replaces the explicit block_ptr / cols that
 * constraint_functions.node_column_blocks builds for the reference's Ip_c column space
 * (constraint_functions.py:112-151: every column except dz[:, :, reference_epoch]). */
int lsq_set_column_blocks_affine(lsq_handle* h, int64_t n_blocks, int32_t k, const int64_t* base, const int64_t* stride,
                                 const int64_t* full_base, const int64_t* full_stride);

int lsq_shape(lsq_handle* h, int64_t* m, int64_t* n, int64_t* nnz);
/* Download the formed A (selected rows only, in row order; canonical CSR, sorted columns). */
int lsq_get_csr(lsq_handle* h, int64_t* indptr, int32_t* indices, double* data);
/* Full CSR of a lazily formed system.  lsq_set_matrix_stencil on one GPU stores only the data rows
 * of G (the stencil rows live as part descriptors); these calls form the full G and Gᵀ on the
 * device and keep them: lsq_get_csr, lsq_spmv / lsq_spmv_rows past the data rows, the dense
 * (precond 2) and band (precond 5) factors, lsq_cov_band*, the mixed multigrid set-up, the
 * assembled SELL operator (precond 0/1 LSQR without the stencil operator) and the distributed
 * relabelling.  lsq_shape does not.  lsq_release_full_csr frees G / Gᵀ / the SELL copies again
 * (the factors already built stay valid); *released = 0 when there was nothing to free (formed
 * eagerly, never expanded, or relabelled for ranks). */
int lsq_release_full_csr(lsq_handle* h, int32_t* released);

/* ---- solve and products ----------------------------------------------------------------- */
/* x = argmin || A x - diag(row_weight)·mask·b ||.  b has length m (unweighted rhs, all rows);
 * x_inout has length n (compacted columns).  Returns 0 converged, 1 maxit reached. */
int lsq_solve(lsq_handle* h, const double* b, double* x_inout, const lsq_opts* o, lsq_stats* s);

/* y = G x (trans = 0; x length n, y length m, UNWEIGHTED rows, all rows) or
 * y = Gᵀ x (trans = 1).  G is the formed operator before row weights and row mask. */
int lsq_spmv(lsq_handle* h, int32_t trans, const double* x, double* y);
/* Rows [first, first + count) of G x only (e.g. the data rows: z_est / residuals, smooth_fit.py:146
 * and :662, without moving the constraint rows over PCIe). */
int lsq_spmv_rows(lsq_handle* h, int64_t first, int64_t count, const double* x, double* y);

/* Output statistics of smooth_fit's parse_model (smooth_fit.py:318-347) without moving the
 * operator to the host.  lsq_rows_sumsq: for each row range k, u = (G x) over rows
 * [first[k], first[k] + count[k]) (x in compacted columns) and sum_w[k] = Σ (w_i u_i)², sum_u[k]
 * = Σ u_i² with w the current row weights (R and RMS of each constraint type, smooth_fit.py:
 * 324-331).  lsq_data_colsum: out = G_dataᵀ f over the FULL column space (length n_full; f has
 * one value per data row, unweighted rows, removed columns included) — the per-node sums of the
 * count / misfit maps (smooth_fit.py:341-347); structured systems on one (y, x) lattice only. */
int lsq_rows_sumsq(lsq_handle* h, const double* x, int32_t n_ranges, const int64_t* first, const int64_t* count,
                   double* sum_w, double* sum_u);
int lsq_data_colsum(lsq_handle* h, const double* f, double* out);

/* Bench / profiling hook: run exactly `iters` LSQR iterations on the current system (no early
 * stop), starting from the state left by the previous call (first call initialises from b).
 * Times only the device iterations. */
int lsq_iterate(lsq_handle* h, const double* b, int64_t iters, const lsq_opts* o, lsq_stats* s);

/* ---- error propagation (replaces sparseqr.rz + inv_tr_upper + row RSS, smooth_fit.py:212-253)
 * Dense device Cholesky AᵀA = RᵀR of the current weighted, masked A (n up to a few 10^4):
 * lsq_sigma_x: E_j = sqrt(diag((AᵀA)^-1))_j = sqrt(row sums of R^-1 squared), length n;
 * lsq_get_rinv: R^-1 as a dense n x n row-major upper-triangular matrix. */
int lsq_sigma_x(lsq_handle* h, double* E);
int lsq_get_rinv(lsq_handle* h, double* Rinv);
/* Column order for precond 5 (band factor): perm[j] = the compact column at position j, chosen so
 * that AᵀA is banded (a grid system: its natural row-major order; others: e.g. reverse
 * Cuthill-McKee).  nullptr = natural order.  Precond 5 (LSQR on the assembled operator,
 * single GPU): M = P·S·R̃⁻¹ with R̃ the banded Cholesky factor of the equilibrated S·PᵀAᵀAP·S
 * (band.hip), applied by one band back / forward substitution per product — the large-n
 * counterpart of precond 2, for systems column scaling cannot precondition (the anisotropic
 * notebook: > 5·10⁴ column-scaled iterations).  Refused when the band is wider than 300 tiles. */
int lsq_set_band_order(lsq_handle* h, int64_t n, const int32_t* perm);

/* Error propagation without a dense factor (replaces sparseqr.rz + inv_tr_upper +
 * propagate_qz_errors at smooth_fit.py:218-253 and op.grid_error(Ip_c·Rinv) at :266-270).
 * perm (length n, nullable = identity): new position j -> compact column perm[j]; an order in
 * which AᵀA is banded (smooth_fit: node-major).  AᵀA of the current weighted, masked system is
 * equilibrated and factored inside its band (64×64 tiles, f64 MFMA); the rows of R⁻¹ needed are
 * formed by banded forward sweeps (never stored).  E[c] = sqrt(((AᵀA)⁻¹)_cc) per compact column.
 * For the n_ops rows of the CSR op (op_ptr[n_ops+1], op_col = compact columns, op_val):
 * op_err[i] = sqrt(op_i (AᵀA)⁻¹ op_iᵀ).  info (nullable, 6): band width in 64-column tiles, tile
 * rows, device bytes, 64×64 tile products of the sweeps, µs of the factorization and of the
 * sweeps (host wall clock).  Error -2 when the band does not fit the device's free memory. */
int lsq_cov_band(lsq_handle* h, const int32_t* perm, double* E, int64_t n_ops, const int64_t* op_ptr,
                 const int32_t* op_col, const double* op_val, double* op_err, int64_t* info);

/* The same for a WINDOW of the columns (compute_E at scale, lssurf_amd/errors.py method 'window'):
 * perm[0..n_win) lists the window's compact columns in a banded order; the principal submatrix
 * (AᵀA)_WW = A_WᵀA_W (the other columns held fixed) is factored and E[j] = sqrt(((AᵀA)_WW⁻¹)_jj)
 * in WINDOW order (n_win entries).  inner (nullable = every position): only the 64-column tiles
 * of the window order that hold a flagged position are swept (the interior whose σ the caller
 * keeps — the margin's sweeps are most of the work), and E is 0 at the other positions.  op rows
 * must lie inside the window.  (AᵀA)⁻¹'s correlations decay with node distance, so the window's
 * interior nodes carry diag((AᵀA)⁻¹) to a tolerance set by the margin (DESIGN.md §Error
 * propagation). */
int lsq_cov_band_window(lsq_handle* h, const int32_t* perm, int64_t n_win, const uint8_t* inner, double* E,
                        int64_t n_ops, const int64_t* op_ptr, const int32_t* op_col, const double* op_val,
                        double* op_err, int64_t* info);

/* Many windows at once (compute_E at scale): window w is perm[win_ptr[w] .. win_ptr[w+1]) with its
 * inner flags and E (window order) at the same positions, and the op rows [win_ops[w],
 * win_ops[w+1]) of the CSR op (op_ptr, op_pos = POSITIONS in window w, op_val; win_ops nullable:
 * none) with op_err per row.  Windows are independent: they run on LSQ_E_LANES (default 2) stream
 * lanes, one window's factorization (a latency-bound chain of tile steps) beside another's sweeps.
 * info (nullable, 6): widest band, most tile rows, device bytes, tile products, µs, lanes. */
int lsq_cov_band_windows(lsq_handle* h, int64_t n_windows, const int64_t* win_ptr, const int32_t* perm,
                         const uint8_t* inner, double* E, const int64_t* win_ops, const int64_t* op_ptr,
                         const int32_t* op_pos, const double* op_val, double* op_err, int64_t* info);

/* Many windows with their bottom margin eliminated first (compute_E at scale; DESIGN.md §Error
 * propagation, round 6): window w's columns are perm[win_ptr[w] .. win_ptr[w+1]) = A = [top margin
 * rows, interior rows] in ascending band order, its last nib[w] columns being Ib (the interior rows
 * the bottom margin's rows reach); bot_perm[bot_ptr[w] .. bot_ptr[w+1]) = B' = the band order of
 * [Ib, bottom margin] REVERSED (bot_ptr[w+1] = bot_ptr[w]: no bottom margin).  B' is factored, its
 * trailing Ib block gives the bottom margin's Schur complement onto Ib, which replaces A's (Ib, Ib)
 * block; A is then factored and swept over the tiles holding an inner position, so the sweeps end
 * at the interior.  E (window order, A's positions) equals lsq_cov_band_windows' E of the whole
 * window [A, bottom margin] to rounding.  Fails (-3, "a deeper Ib is needed") when a row holds a
 * column of A outside Ib and one of the bottom margin.  info as lsq_cov_band_windows. */
int lsq_cov_band_windows_schur(lsq_handle* h, int64_t n_windows, const int64_t* win_ptr, const int32_t* perm,
                               const uint8_t* inner, double* E, const int64_t* bot_ptr, const int32_t* bot_perm,
                               const int64_t* nib, int64_t* info);

/* The banded factor itself (replaces sparseqr.rz's R and E, smooth_fit.py:218 / the aniso notebook):
 * for the current weighted, masked A and the column order perm (nullable = natural),
 * (A·P)ᵀ(A·P) = RᵀR with R = R̃·S⁻¹, R̃ the upper band factor of the equilibrated S·Pᵀ(AᵀA)P·S.
 * info (3): n, T = tile rows (n padded to 64·T), w = tiles right of the diagonal per tile row.  When
 * R is non-null: R̃ as T·(w+1) row-major 64×64 tiles, tile (I, J) (I ≤ J ≤ I + w) at
 * (I·(w+1) + J − I)·4096 (use the upper triangle of diagonal tiles), sc = diag(S) (64·T), perm_out =
 * P (new position -> compact column, n).  Call once with R = NULL for the sizes.  -5 when the band
 * does not fit the device. */
int lsq_band_factor(lsq_handle* h, const int32_t* perm, int64_t* info, double* R, double* sc, int32_t* perm_out);

/* ---- multi-GPU (one process per GPU) --------------------------------------
 * lsq_dist_unique_id: rank 0 creates the 128-byte RCCL id; the caller broadcasts it (any
 * transport); every rank then calls lsq_create_dist.  Each rank forms only the rows it owns
 * (lsq_set_col_map + lsq_set_matrix_* with GLOBAL column ids), reads which columns its rows
 * reference, and installs its layout: col_local maps every global column to a local id
 * ([0, n_own) owned, [n_own, n_local) ghosts grouped by owning peer, -1 unused); for each
 * peer, send_idx lists the owned local columns that peer holds as ghosts (in the order of the
 * peer's ghost slots) and recv_cnt the number of ghosts it owns.  lsq_solve / lsq_iterate then
 * run one LSQR over all ranks: halo exchange of ghost v before A·v, reverse halo of ghost
 * partial sums after Aᵀu, RCCL all-reduce of the scalar norms; x_inout receives the owned
 * columns (length n_own). */
int lsq_dist_unique_id(uint8_t* id128);
lsq_handle* lsq_create_dist(int32_t device, int32_t rank, int32_t nranks, const uint8_t* id128);
/* What the rank's RCCL communicator and device report (bench.py's self-check of a multi-GPU run):
 * out[0] ncclCommCount, out[1] ncclCommUserRank, out[2] ncclCommCuDevice, out[3] the handle's
 * HIP device, out[4..6] its PCI domain / bus / device ids (a physical card: two ranks with equal
 * ids share one GPU).  A handle without a communicator reports count 0. */
int lsq_dist_comm_info(lsq_handle* h, int64_t* out7);
int lsq_dist_referenced_cols(lsq_handle* h, uint8_t* flags);
int lsq_dist_set_layout(lsq_handle* h, const int32_t* col_local, int64_t n_local, int64_t n_own,
                        int32_t n_peers, const int32_t* peers, const int64_t* send_cnt,
                        const int32_t* send_idx, const int64_t* recv_cnt);

/* Structured-operator ranks (systems formed by lsq_set_matrix_stencil): each rank forms its
 * window of node rows — owned rows ± halo rows, as sub-grids with their own column numbering —
 * and installs the halo: own_ranges = n_ranges [start, end) pairs of owned local full columns;
 * per peer, send_idx lists owned local columns that peer holds as ghosts and recv_idx the local
 * ghost columns that peer owns (both in ascending GLOBAL column order).  lsq_solve then returns
 * every local compact column in x_inout (length = the local compact width; ghosts come out 0). */
int lsq_dist_set_halo(lsq_handle* h, int32_t n_ranges, const int64_t* own_ranges, int32_t n_peers,
                      const int32_t* peers, const int64_t* send_cnt, const int32_t* send_idx,
                      const int64_t* recv_cnt, const int32_t* recv_idx);

/* Multigrid over ranks (precond 4, method 1): the global structure behind a structured rank's
 * window — the global grids and stencil parts (the descriptors of lsq_set_matrix_stencil for the
 * whole system; field-valued parts with ntpl = 0), local_of[s] = the rank's stencil index of global
 * stencil s (-1: the rank holds none of its rows), and the window in global node rows of dim 0:
 * window start, owned rows [own_row0, own_row1), rows of the lattice.  Level 0 of the V-cycle is
 * each rank's window (halo exchanges around every operator application), the coarse levels are
 * the global Galerkin levels replicated on every rank (the restricted residual summed over the
 * ranks once per cycle, the lumped data rows once per solve). */
int lsq_dist_set_global(lsq_handle* h, int64_t n_full, int32_t n_grids, const lsq_grid_desc* grids, int32_t n_stencil,
                        const lsq_stencil_desc* stencils, const int32_t* local_of, int32_t win_row0, int32_t own_row0,
                        int32_t own_row1, int32_t rows);

/* Virtual ranks: the same distributed solve with every rank of the partition in THIS process
 * on one device (exchanges become device copies).  Configure each rank's handle exactly as a
 * real rank (lsq_set_col_map, lsq_set_matrix_*, lsq_dist_referenced_cols,
 * lsq_dist_set_layout), then solve all ranks at once; b / x are per-rank arrays. */
typedef struct lsq_vgroup lsq_vgroup;
lsq_vgroup* lsq_vgroup_create(int32_t device, int32_t nranks);
lsq_handle* lsq_vgroup_rank(lsq_vgroup* g, int32_t rank);
int lsq_vgroup_solve(lsq_vgroup* g, const double* const* b, double* const* x, const lsq_opts* o,
                     lsq_stats* s);
int lsq_vgroup_iterate(lsq_vgroup* g, const double* const* b, int64_t iters, const lsq_opts* o,
                       lsq_stats* s);
const char* lsq_vgroup_last_error(lsq_vgroup* g);
void lsq_vgroup_destroy(lsq_vgroup* g);

/* Device group: the distributed solve over N distinct devices from ONE process (smooth_fit's
 * n_gpus; SURVEY.md §8(b) "ranks invisible to Python").  One RCCL communicator per device
 * (ncclCommInitAll); each solve runs every rank on its own host thread with the kernels, halos
 * and all-reduces of a one-process-per-GPU rank.  Configure each rank's handle as a real rank
 * (lsq_set_col_map, lsq_set_matrix_stencil, lsq_dist_set_halo, lsq_dist_set_global ...).
 * Repeated devices are refused (NULL): one device runs the same ranks through lsq_vgroup. */
typedef struct lsq_dgroup lsq_dgroup;
lsq_dgroup* lsq_dgroup_create(int32_t n, const int32_t* devices);
lsq_handle* lsq_dgroup_rank(lsq_dgroup* g, int32_t rank);
int lsq_dgroup_solve(lsq_dgroup* g, const double* const* b, double* const* x, const lsq_opts* o, lsq_stats* s);
int lsq_dgroup_iterate(lsq_dgroup* g, const double* const* b, int64_t iters, const lsq_opts* o,
                       lsq_stats* s);
const char* lsq_dgroup_last_error(lsq_dgroup* g);
void lsq_dgroup_destroy(lsq_dgroup* g);
/* The rank threads of a device-group call meet at a host fence before every RCCL call; a rank
 * that fails poisons it, so the others return an error at their next collective instead of
 * blocking in it.  Self-test of that fence (no device): n threads pass `rounds` fences, thread
 * fail_rank (-1: none) throws before round fail_rank; returns the number of threads that left
 * on the poisoned fence (n - 1 when one rank failed, 0 otherwise). */
int lsq_fence_selftest(int32_t n, int32_t fail_rank, int32_t rounds);

/* ---- outlier editing (RDE.py:10-18, calc_sigma_extra.py:13-44) -----
 * calc_sigma_extra's bounded search evaluates RDE(r / sqrt(s² + σ²)) 25–30 times per outer
 * iteration.  lsq_rde_create uploads r and σ once (finite entries only); lsq_rde_order_stats
 * returns the requested order statistics (0-based ranks) of r / sqrt(s² + σ²), computed exactly
 * as numpy does, so the caller's percentile interpolation is bit-identical to RDE's. */
typedef struct lsq_rde lsq_rde;
lsq_rde* lsq_rde_create(int32_t device, int64_t n, const double* r, const double* sigma);
int lsq_rde_order_stats(lsq_rde* c, double sigma_extra, int64_t n_idx, const int64_t* idx, double* out);
const char* lsq_rde_last_error(lsq_rde* c);
void lsq_rde_destroy(lsq_rde* c);

/* Bench / profiling hooks.  lsq_profile_kernels times each iteration kernel of the operator
 * `op` (lsq_opts.op) in isolation (reps launches each, HIP events on the handle's stream):
 * out8 = {ms of x/w+A·v, ms of Aᵀu, ms of beta reduce, ms of rotation, algorithmic HBM bytes
 * per launch of x/w+A·v, of Aᵀu (DESIGN.md §Byte model), 0, 0}.  It clobbers the iteration
 * state.  lsq_sell_info: out8 = {m, n, nnz, SELL entries streamed by A·v, by Aᵀu, device bytes
 * of the operator copies, 1 if the structured stencil operator is available, n_full}. */
int lsq_profile_kernels(lsq_handle* h, int32_t reps, int32_t op, double* out8);
/* CGNR (method 1) hooks.  lsq_cg_available: 1 when method 1 runs CGNR on this system with this
 * preconditioner (it builds the normal-stencil tables), 0 when it would fall back to LSQR (the
 * reason is in lsq_last_error).  lsq_profile_cg: per-kernel HIP-event times of one CG iteration,
 * out8 = {ms data rows t = Ad·p, ms normal operator q = N p + Adᵀt, ms update + preconditioner,
 * ms of the two scalar kernels, algorithmic HBM bytes per launch of the first three, 0}.
 * lsq_normal_apply: q = AᵀA p for the current row weights/mask, p and q over the FULL column
 * space (length n_full of lsq_set_col_map; test hook for the normal operator). */
int lsq_cg_available(lsq_handle* h, int32_t precond);
int lsq_profile_cg(lsq_handle* h, int32_t reps, int32_t precond, double* out8);
/* Multigrid (precond 4) test hooks.  lsq_mg_info: out[0] = levels L, then per level
 * (S0, S1, n_full, removed epoch) — cap must hold 1 + 4L values; with room for 2 + 4L, out[1 + 4L] =
 * the first level of the one-workgroup tail V-cycle (k_mg_tail), −1 for none.  lsq_mg_apply on level l's full
 * column space (z0 grid then dz grid, in the system's order): what 0: y = N_l x (level 0: AᵀA;
 * coarse levels: Galerkin PᵀNP of the stencil rows + the (y, x)-lumped data rows), 1: y = the
 * V-cycle applied to x (level 0), 2: y[0] = the smoother's λ_max(M⁻¹N) estimate of level l.
 * Both build the hierarchy for the current row weights / mask. */
int lsq_mg_info(lsq_handle* h, int64_t* out, int64_t cap);
int lsq_mg_apply(lsq_handle* h, int32_t level, int32_t what, const double* x, double* y);
int lsq_normal_apply(lsq_handle* h, const double* p, double* q);
int lsq_sell_info(lsq_handle* h, int64_t* out8);

/* ---- triangular kernels (replace the Cython kernels; R upper triangular CSR, int32 indices,
 *      sorted column indices, diagonal first in each row) ------------------------------------ */
/* spsolve_tr_upper: x = R^-1 b. */
int tri_upper_solve_csr(int32_t device, int64_t N, const int32_t* indptr, const int32_t* indices,
                        const double* data, const double* b, double* x);
/* inv_tr_upper: columns col = N-1..0 of R^-1, entries emitted (col descending, row descending)
 * when row == col or |x| > tol (tol is a C float, as in the .pyx).  Returns 1 (buffer full)
 * exactly when inv_tr_upper returns status 1, with the same nnz_max entries in rr/cc/vv (the
 * last one zero).  *n_out = number of entries written. */
int tri_upper_inv_csr(int32_t device, int64_t N, const int32_t* indptr, const int32_t* indices,
                      const double* data, int64_t nnz_max, float tol,
                      int32_t* rr, int32_t* cc, double* vv, int64_t* n_out);
/* propagate_qz_errors: E_i = sqrt(sum over columns of (R^-1)_{i,col}^2). */
int tri_upper_rowrss_csr(int32_t device, int64_t N, const int32_t* indptr, const int32_t* indices,
                         const double* data, double* E);
/* Error string of the last failing tri_* call on this thread. */
const char* tri_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* LSQSURF_H */
