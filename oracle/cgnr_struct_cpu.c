/* cgnr_struct_cpu.c — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
 *
 * The second kind of bench.py's CPU baseline (VERDICT r4 Weak #5 / Next #8): the same CGNR +
 * block-Jacobi as cgnr_cpu.c, but on the STRUCTURED operator the GPU line uses instead of an
 * assembled CSR — no stored matrix:
 *   stencil rows  from the part descriptors (lsq_stencil_desc: grid, centre box, template offsets
 *                 and values; lin_op.py:80-132, the constraint rows of smooth_fit.py:591-627): the
 *                 row of centre c is  rs_r · Σ_t val_t · p[c + off_t];
 *   data rows     matrix-free from the points' float subscripts f_d = (p_d − b0_d)/δ_d (the
 *                 numbers lin_op.interp_mtx, lin_op.py:163-247, derives its bilinear / trilinear
 *                 weights from, ((1·w_y)·w_x)·w_t), the points sorted by (y, x) cell so Aᵀ gathers
 *                 per node over the ≤ 4 cells around it (deterministic, no atomics);
 * both of the form A = diag(rs)·G·Ip_c, rs = the row weights × the row mask.  As on the GPU, the
 * vectors live in the FULL column space (columns removed by Ip_c hold 0).  One iteration:
 * t = A p (a pass over every row), γ = ‖t‖², q = Aᵀt (a gather per node), then cgnr_cpu.c's update.
 * Same iterates as the CSR kind up to the summation order (tests/test_oracle_cgnr.py).  Requires the
 * interpolation grids to share one (y, x) lattice (every smooth_fit system with equal z0 / dz
 * spacing — the GPU's matrix-free data rows have the same condition); returns −2 otherwise.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KB 16
#define MAXG 4

typedef struct {   /* = lsq_grid_desc (include/lsqsurf.h) */
    int32_t ndim, reserved;
    int64_t shape[3];
    int64_t col0;
    double b0[3], delta[3];
} GridD;
typedef struct {   /* = lsq_stencil_desc */
    int32_t grid, ntpl;
    int32_t off[8][3];
    double val[8];
    int64_t row0, n_eq;
    int64_t lo[3], hi[3];
} PartD;

typedef struct {
    int ng, np;
    const GridD* g;
    const PartD* p;
    int64_t S[MAXG][3];           /* grid shapes, 1 past ndim */
    int64_t npts, m, n_full;
    const double* rs;
    uint8_t* kept;                /* full column kept by Ip_c */
    /* interpolation: 2-D grids (z0) and at most one 3-D grid (dz) on one (y, x) lattice */
    int n2, g2[MAXG], g3, isinterp[MAXG];
    int64_t S0, S1, S2;
    /* points sorted by cell: cell subscripts, fractions, row scale, original row */
    int32_t *cy, *cx, *ct;
    double *fy, *fx, *ft, *prs;
    int64_t* pidx;
    int64_t* cptr;                /* cell (cy·(S1−1) + cx) -> first sorted point; ncell + 1 */
    int64_t* blkof;               /* full column -> block·KB + position in it (−1: none) */
} Op;

static void cell_frac(double f, int64_t S, int32_t* c, double* fr) {
    double cf = floor(f);
    if (cf > (double)(S - 2) || cf < 0.0) cf = cf < 0.0 ? 0.0 : (double)(S - 2);
    *c = (int32_t)cf;
    *fr = f - cf;   /* f = S − 1: cell S − 2, fraction 1 — the weights k_gen_rows gives node S − 1 */
}

/* A value of sorted point s on node (y, x) [epoch t of the 3-D grid; t < 0: a 2-D grid], 0 when
 * the point does not touch it: ((1·w_y)·w_x)·w_t · rs as lin_op.interp_mtx + toCSR's row weight */
static inline double pt_weight(const Op* o, int64_t s, int64_t y, int64_t x, int64_t t) {
    double w = 1.0;
    if (y == o->cy[s]) w *= 1.0 - o->fy[s];
    else if (y == o->cy[s] + 1) w *= o->fy[s];
    else return 0.0;
    if (x == o->cx[s]) w *= 1.0 - o->fx[s];
    else if (x == o->cx[s] + 1) w *= o->fx[s];
    else return 0.0;
    if (t >= 0) {
        if (t == o->ct[s]) w *= 1.0 - o->ft[s];
        else if (t == o->ct[s] + 1) w *= o->ft[s];
        else return 0.0;
    }
    return w * o->prs[s];
}

/* grid of full column f and its subscripts; −1 outside every grid */
static int decode(const Op* o, int64_t f, int64_t sub[3]) {
    for (int g = 0; g < o->ng; ++g) {
        const int64_t r0 = f - o->g[g].col0, n = o->S[g][0] * o->S[g][1] * o->S[g][2];
        if (r0 < 0 || r0 >= n) continue;
        sub[2] = r0 % o->S[g][2];
        sub[1] = (r0 / o->S[g][2]) % o->S[g][1];
        sub[0] = r0 / (o->S[g][2] * o->S[g][1]);
        return g;
    }
    return -1;
}

static inline int64_t col_of(const Op* o, int g, int64_t y, int64_t x, int64_t t) {
    return o->g[g].col0 + (y * o->S[g][1] + x) * o->S[g][2] + t;
}

/* linear offset of template t of part P in its grid; extent of its row box (1 past ndim) */
static int64_t tpl_col(const Op* o, const PartD* P, int t) {
    const int64_t* S = o->S[P->grid];
    return ((int64_t)P->off[t][0] * S[1] + P->off[t][1]) * S[2] + P->off[t][2];
}
static void box_ext(const Op* o, const PartD* P, int64_t E[3]) {
    const int nd = o->g[P->grid].ndim;
    for (int d = 0; d < 3; ++d) E[d] = d < nd ? P->hi[d] - P->lo[d] : 1;
}

/* t = A p (p in the full space, 0 on removed columns): data rows (sorted point order) into td,
 * stencil rows into tr (row − npts) */
static void op_fwd(const Op* o, const double* p, double* td, double* tr) {
#pragma omp parallel for schedule(static)
    for (int64_t s = 0; s < o->npts; ++s) {
        const double fr[3] = {o->fy[s], o->fx[s], o->ft[s]};
        double acc = 0.0;
        for (int k = 0; k < o->n2 + (o->g3 >= 0); ++k) {
            const int g = k < o->n2 ? o->g2[k] : o->g3;
            const int nd = o->g[g].ndim;
            for (int q = 0; q < (1 << nd); ++q) {
                double w = 1.0;
                int64_t c[3] = {o->cy[s], o->cx[s], nd == 3 ? o->ct[s] : 0};
                for (int d = 0; d < nd; ++d) {
                    const int bit = (q >> (nd - 1 - d)) & 1;
                    c[d] += bit;
                    w *= bit ? fr[d] : (1.0 - fr[d]);
                }
                if (w != 0.0) acc += (w * o->prs[s]) * p[col_of(o, g, c[0], c[1], c[2])];
            }
        }
        td[s] = acc;
    }
    for (int s = 0; s < o->np; ++s) {
        const PartD* P = o->p + s;
        const int g = P->grid;
        int64_t E[3], off[8];
        box_ext(o, P, E);
        for (int t = 0; t < P->ntpl; ++t) off[t] = tpl_col(o, P, t);
        const int64_t lo2 = o->g[g].ndim == 3 ? P->lo[2] : 0, lo1 = o->g[g].ndim >= 2 ? P->lo[1] : 0;
        double* trp = tr + (P->row0 - o->npts);
        const double* rsp = o->rs + P->row0;
#pragma omp parallel for schedule(static)
        for (int64_t a = 0; a < E[0]; ++a)
            for (int64_t b = 0; b < E[1]; ++b) {
                const int64_t k0 = (a * E[1] + b) * E[2];
                const int64_t c0 = col_of(o, g, P->lo[0] + a, lo1 + b, lo2);
                for (int64_t c = 0; c < E[2]; ++c) {
                    const double w = rsp[k0 + c];
                    double acc = 0.0;
                    for (int t = 0; t < P->ntpl; ++t)
                        if (P->val[t] != 0.0) acc += (w * P->val[t]) * p[c0 + c + off[t]];
                    trp[k0 + c] = acc;
                }
            }
    }
}

/* q = Aᵀ t over the full space (removed columns: 0), one gather per (y, x) node */
static void op_adj(const Op* o, const double* td, const double* tr, double* q) {
    const int64_t C1 = o->S1 - 1;
    for (int g = 0; g < o->ng; ++g) {
        const int64_t S0 = o->S[g][0], S1 = o->S[g][1], S2 = o->S[g][2];
        const int nd = o->g[g].ndim;
#pragma omp parallel for schedule(static)
        for (int64_t y = 0; y < S0; ++y)
            for (int64_t x = 0; x < S1; ++x) {
                double acc[64];
                for (int64_t t = 0; t < S2; ++t) acc[t] = 0.0;
                if (o->isinterp[g]) {   /* data rows: the points of the ≤ 4 cells around the node */
                    for (int64_t cy = y - 1; cy <= y; ++cy)
                        for (int64_t cx = x - 1; cx <= x; ++cx) {
                            if (cy < 0 || cy > o->S0 - 2 || cx < 0 || cx > o->S1 - 2) continue;
                            for (int64_t s = o->cptr[cy * C1 + cx]; s < o->cptr[cy * C1 + cx + 1]; ++s) {
                                if (nd == 3) {
                                    const int64_t c = o->ct[s];
                                    acc[c] += pt_weight(o, s, y, x, c) * td[s];
                                    acc[c + 1] += pt_weight(o, s, y, x, c + 1) * td[s];
                                } else {
                                    acc[0] += pt_weight(o, s, y, x, -1) * td[s];
                                }
                            }
                        }
                }
                for (int s = 0; s < o->np; ++s) {   /* stencil rows: centres c − off_t in the box */
                    const PartD* P = o->p + s;
                    if (P->grid != g) continue;
                    int64_t E[3];
                    box_ext(o, P, E);
                    const int64_t lo1 = nd >= 2 ? P->lo[1] : 0, lo2 = nd == 3 ? P->lo[2] : 0;
                    const double* trp = tr + (P->row0 - o->npts);
                    const double* rsp = o->rs + P->row0;
                    for (int tp = 0; tp < P->ntpl; ++tp) {
                        if (P->val[tp] == 0.0) continue;
                        const int64_t a = y - P->off[tp][0] - P->lo[0], b = x - P->off[tp][1] - lo1;
                        if (a < 0 || a >= E[0] || b < 0 || b >= E[1]) continue;
                        const int64_t k0 = (a * E[1] + b) * E[2];
                        for (int64_t t = 0; t < S2; ++t) {
                            const int64_t c = t - P->off[tp][2] - lo2;
                            if (c < 0 || c >= E[2]) continue;
                            acc[t] += (rsp[k0 + c] * P->val[tp]) * trp[k0 + c];
                        }
                    }
                }
                const int64_t c0 = col_of(o, g, y, x, 0);
                for (int64_t t = 0; t < S2; ++t) q[c0 + t] = o->kept[c0 + t] ? acc[t] : 0.0;
            }
    }
}

static double dot(int64_t n, const double* a, const double* b) {
    double s = 0.0;
#pragma omp parallel for reduction(+ : s) schedule(static)
    for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}

/* position of full column f in block bb (−1: not in it) */
static inline int in_block(const Op* o, int64_t bb, int64_t f) {
    const int64_t e = o->blkof[f];
    return e >= 0 && e / KB == bb ? (int)(e % KB) : -1;
}

/* Σ v_a v_b over a row's block values v (a ≤ b) into Rb (upper, row-major KB×KB) */
static void add_pairs(const double* v, int k, double* Rb) {
    for (int a = 0; a < k; ++a) {
        if (v[a] == 0.0) continue;
        for (int b = a; b < k; ++b)
            if (v[b] != 0.0) Rb[a * KB + b] += v[a] * v[b];
    }
}

/* (AᵀA)_bb of block bb (full column ids fb[0..k)) from the rows touching its columns, each row
 * once: the data rows of the union of the cells around the block's nodes, the stencil rows from
 * the first block column they touch */
static void block_normal(const Op* o, int64_t bb, const int64_t* fb, int k, double* Rb) {
    const int64_t C1 = o->S1 - 1;
    int64_t sb[KB][3];
    int gb[KB];
    for (int a = 0; a < k; ++a) gb[a] = decode(o, fb[a], sb[a]);
    double v[KB];
    int64_t cells[4 * KB];
    int nc = 0;
    for (int a = 0; a < k; ++a) {
        if (gb[a] < 0 || !o->isinterp[gb[a]]) continue;
        for (int64_t cy = sb[a][0] - 1; cy <= sb[a][0]; ++cy)
            for (int64_t cx = sb[a][1] - 1; cx <= sb[a][1]; ++cx) {
                if (cy < 0 || cy > o->S0 - 2 || cx < 0 || cx > o->S1 - 2) continue;
                const int64_t cell = cy * C1 + cx;
                int seen = 0;
                for (int l = 0; l < nc; ++l) seen |= cells[l] == cell;
                if (!seen) cells[nc++] = cell;
            }
    }
    for (int l = 0; l < nc; ++l)
        for (int64_t s = o->cptr[cells[l]]; s < o->cptr[cells[l] + 1]; ++s) {
            for (int a = 0; a < k; ++a)
                v[a] = gb[a] >= 0 && o->isinterp[gb[a]]
                           ? pt_weight(o, s, sb[a][0], sb[a][1], o->g[gb[a]].ndim == 3 ? sb[a][2] : -1)
                           : 0.0;
            add_pairs(v, k, Rb);
        }
    for (int i = 0; i < k; ++i) {
        const int g = gb[i];
        if (g < 0) continue;
        const int nd = o->g[g].ndim;
        for (int s = 0; s < o->np; ++s) {   /* stencil rows through column i */
            const PartD* P = o->p + s;
            if (P->grid != g) continue;
            int64_t E[3];
            box_ext(o, P, E);
            for (int t1 = 0; t1 < P->ntpl; ++t1) {
                if (P->val[t1] == 0.0) continue;
                int64_t c[3] = {0, 0, 0}, kr = 0;
                int in = 1;
                for (int d = 0; d < 3; ++d) {
                    const int64_t lo = d < nd ? P->lo[d] : 0;
                    c[d] = sb[i][d] - P->off[t1][d];
                    in = in && c[d] >= lo && c[d] < lo + E[d];
                    kr = kr * E[d] + (c[d] - lo);
                }
                if (!in) continue;
                const double w = o->rs[P->row0 + kr];
                for (int a = 0; a < k; ++a) v[a] = 0.0;
                for (int t2 = 0; t2 < P->ntpl; ++t2) {
                    if (P->val[t2] == 0.0) continue;
                    const int l = in_block(o, bb, col_of(o, g, c[0] + P->off[t2][0], c[1] + P->off[t2][1],
                                                         c[2] + P->off[t2][2]));
                    if (l >= 0) v[l] += w * P->val[t2];
                }
                int first = 1;
                for (int a = 0; a < i; ++a) first &= v[a] == 0.0;
                if (first) add_pairs(v, k, Rb);
            }
        }
    }
}

static int op_init(Op* o, int32_t n_grids, const GridD* grids, int32_t n_interp, const int32_t* interp_grid,
                   int64_t npts, const double* py, const double* px, const double* pt, int32_t n_parts,
                   const PartD* parts, int64_t m, int64_t n_full, const double* rs, int64_t n, const int64_t* keep) {
    memset(o, 0, sizeof(*o));
    if (n_grids < 1 || n_grids > MAXG || n_interp < 1) return -2;
    o->ng = n_grids;
    o->g = grids;
    o->np = n_parts;
    o->p = parts;
    o->npts = npts;
    o->m = m;
    o->rs = rs;
    o->n_full = n_full;
    o->g3 = -1;
    for (int g = 0; g < n_grids; ++g)
        for (int d = 0; d < 3; ++d) o->S[g][d] = d < grids[g].ndim ? grids[g].shape[d] : 1;
    for (int s = 0; s < n_parts; ++s)
        if (parts[s].grid < 0 || parts[s].grid >= n_grids || parts[s].ntpl > 8) return -2;
    const GridD* L = grids + interp_grid[0];
    for (int k = 0; k < n_interp; ++k) {
        const GridD* G = grids + interp_grid[k];
        if (G->ndim < 2 || G->shape[0] != L->shape[0] || G->shape[1] != L->shape[1] || G->b0[0] != L->b0[0] ||
            G->b0[1] != L->b0[1] || G->delta[0] != L->delta[0] || G->delta[1] != L->delta[1])
            return -2;   /* not one (y, x) lattice */
        if (G->ndim == 3) {
            if (o->g3 >= 0) return -2;
            o->g3 = interp_grid[k];
        } else {
            o->g2[o->n2++] = interp_grid[k];
        }
        o->isinterp[interp_grid[k]] = 1;
    }
    for (int g = 0; g < n_grids; ++g)
        if (o->S[g][2] > 64) return -2;
    o->S0 = L->shape[0];
    o->S1 = L->shape[1];
    o->S2 = o->g3 >= 0 ? grids[o->g3].shape[2] : 1;
    if (o->S0 < 2 || o->S1 < 2 || (o->g3 >= 0 && o->S2 < 2)) return -2;
    o->kept = (uint8_t*)calloc(n_full > 0 ? n_full : 1, 1);
    for (int64_t j = 0; j < n; ++j) o->kept[keep[j]] = 1;
    /* points sorted by (y, x) cell (stable counting sort) */
    const int64_t C1 = o->S1 - 1, ncell = (o->S0 - 1) * C1;
    const GridD* T = o->g3 >= 0 ? grids + o->g3 : NULL;
    const int64_t np1 = npts > 0 ? npts : 1;
    int64_t* key = (int64_t*)malloc(sizeof(int64_t) * np1);
    o->cptr = (int64_t*)calloc(ncell + 1, sizeof(int64_t));
    for (int64_t r = 0; r < npts; ++r) {
        int32_t cy, cx;
        double fr;
        cell_frac((py[r] - L->b0[0]) / L->delta[0], o->S0, &cy, &fr);
        cell_frac((px[r] - L->b0[1]) / L->delta[1], o->S1, &cx, &fr);
        key[r] = (int64_t)cy * C1 + cx;
        o->cptr[key[r] + 1]++;
    }
    for (int64_t c = 0; c < ncell; ++c) o->cptr[c + 1] += o->cptr[c];
    int64_t* slot = (int64_t*)malloc(sizeof(int64_t) * (ncell > 0 ? ncell : 1));
    memcpy(slot, o->cptr, sizeof(int64_t) * ncell);
    o->cy = (int32_t*)malloc(sizeof(int32_t) * np1);
    o->cx = (int32_t*)malloc(sizeof(int32_t) * np1);
    o->ct = (int32_t*)calloc(np1, sizeof(int32_t));
    o->fy = (double*)malloc(sizeof(double) * np1);
    o->fx = (double*)malloc(sizeof(double) * np1);
    o->ft = (double*)calloc(np1, sizeof(double));
    o->prs = (double*)malloc(sizeof(double) * np1);
    o->pidx = (int64_t*)malloc(sizeof(int64_t) * np1);
    for (int64_t r = 0; r < npts; ++r) {
        const int64_t s = slot[key[r]]++;
        /* the subscripts as k_gen_rows computes them: one IEEE division per dim */
        cell_frac((py[r] - L->b0[0]) / L->delta[0], o->S0, o->cy + s, o->fy + s);
        cell_frac((px[r] - L->b0[1]) / L->delta[1], o->S1, o->cx + s, o->fx + s);
        if (T) cell_frac((pt[r] - T->b0[2]) / T->delta[2], o->S2, o->ct + s, o->ft + s);
        o->prs[s] = rs[r];
        o->pidx[s] = r;
    }
    free(slot);
    free(key);
    return 0;
}

static void op_free(Op* o) {
    free(o->kept); free(o->cptr); free(o->cy); free(o->cx); free(o->ct); free(o->fy); free(o->fx); free(o->ft);
    free(o->prs); free(o->pidx); free(o->blkof);
}

/* ‖A‖_F² over the kept columns */
static double op_frob2(const Op* o) {
    double s2 = 0.0;
#pragma omp parallel for reduction(+ : s2) schedule(static)
    for (int64_t s = 0; s < o->npts; ++s) {
        const double fr[3] = {o->fy[s], o->fx[s], o->ft[s]};
        for (int k = 0; k < o->n2 + (o->g3 >= 0); ++k) {
            const int g = k < o->n2 ? o->g2[k] : o->g3;
            const int nd = o->g[g].ndim;
            for (int q = 0; q < (1 << nd); ++q) {
                double w = 1.0;
                int64_t c[3] = {o->cy[s], o->cx[s], nd == 3 ? o->ct[s] : 0};
                for (int d = 0; d < nd; ++d) {
                    const int bit = (q >> (nd - 1 - d)) & 1;
                    c[d] += bit;
                    w *= bit ? fr[d] : (1.0 - fr[d]);
                }
                if (w != 0.0 && o->kept[col_of(o, g, c[0], c[1], c[2])]) s2 += (w * o->prs[s]) * (w * o->prs[s]);
            }
        }
    }
    for (int s = 0; s < o->np; ++s) {
        const PartD* P = o->p + s;
        const int g = P->grid, nd = o->g[g].ndim;
        int64_t E[3];
        box_ext(o, P, E);
        const int64_t lo1 = nd >= 2 ? P->lo[1] : 0, lo2 = nd == 3 ? P->lo[2] : 0;
#pragma omp parallel for reduction(+ : s2) schedule(static)
        for (int64_t k = 0; k < P->n_eq; ++k) {
            const int64_t c2 = k % E[2], c1 = (k / E[2]) % E[1], c0 = k / (E[2] * E[1]);
            const double w = o->rs[P->row0 + k];
            for (int t = 0; t < P->ntpl; ++t)
                if (P->val[t] != 0.0 && o->kept[col_of(o, g, P->lo[0] + c0 + P->off[t][0], lo1 + c1 + P->off[t][1],
                                                       lo2 + c2 + P->off[t][2])])
                    s2 += (w * P->val[t]) * (w * P->val[t]);
        }
    }
    return s2;
}

/* stats: [iters, time_s (iterations only), setup_s, threads, snorm, rnorm, anorm_f] (as cgnr_bj_cpu);
 * x: compact columns (keep order) */
int cgnr_bj_struct_cpu(int32_t n_grids, const GridD* grids, int32_t n_interp, const int32_t* interp_grid,
                       int64_t npts, const double* py, const double* px, const double* pt, int32_t n_parts,
                       const PartD* parts, int64_t m, int64_t n_full, const double* rs, int64_t n,
                       const int64_t* keep, const double* b, int64_t nblk, const int64_t* bptr,
                       const int32_t* bcols, double* x, double atol, int64_t maxit, int64_t fixed_iters,
                       int nthreads, double* stats) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
    const double t0 = omp_get_wtime();
    Op o;
    const int rc = op_init(&o, n_grids, grids, n_interp, interp_grid, npts, py, px, pt, n_parts, parts, m, n_full,
                           rs, n, keep);
    if (rc) {
        op_free(&o);
        return rc;
    }
    /* block factors: R_b (upper, row-major k×k) with dead columns zeroed; blocks over full ids */
    double* R = (double*)calloc((size_t)(nblk > 0 ? nblk : 1) * KB * KB, sizeof(double));
    int64_t* fcol = (int64_t*)malloc(sizeof(int64_t) * (bptr[nblk] > 0 ? bptr[nblk] : 1));
    int bad = 0;
    o.blkof = (int64_t*)malloc(sizeof(int64_t) * (n_full > 0 ? n_full : 1));
    for (int64_t f = 0; f < n_full; ++f) o.blkof[f] = -1;
    for (int64_t bb = 0; bb < nblk && !bad; ++bb) {
        if (bptr[bb + 1] - bptr[bb] > KB) bad = 1;
        for (int64_t e = bptr[bb]; e < bptr[bb + 1] && !bad; ++e) {
            fcol[e] = keep[bcols[e]];
            o.blkof[fcol[e]] = bb * KB + (e - bptr[bb]);
        }
    }
    if (bad) {
        free(R); free(fcol);
        op_free(&o);
        return -1;
    }
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t bb = 0; bb < nblk; ++bb) {
        const int64_t b0 = bptr[bb];
        const int k = (int)(bptr[bb + 1] - b0);
        double* Rb = R + bb * KB * KB;
        block_normal(&o, bb, fcol + b0, k, Rb);
        for (int j = 0; j < k; ++j) {   /* Cholesky, upper: N = RᵀR */
            double d = Rb[j * KB + j];
            for (int l = 0; l < j; ++l) d -= Rb[l * KB + j] * Rb[l * KB + j];
            if (!(d > 0.0)) {
                for (int l = j; l < k; ++l) Rb[j * KB + l] = 0.0;
                continue;
            }
            const double r = sqrt(d);
            Rb[j * KB + j] = r;
            for (int i = j + 1; i < k; ++i) {
                double s = Rb[j * KB + i];
                for (int l = 0; l < j; ++l) s -= Rb[l * KB + j] * Rb[l * KB + i];
                Rb[j * KB + i] = s / r;
            }
        }
    }
    const double anorm_f = sqrt(op_frob2(&o));
    const int64_t ms = m - npts, nf = n_full;
    double *s = (double*)calloc(nf, sizeof(double)), *z = (double*)calloc(nf, sizeof(double));
    double *p = (double*)calloc(nf, sizeof(double)), *q = (double*)calloc(nf, sizeof(double));
    double *xf = (double*)calloc(nf, sizeof(double));
    double *td = (double*)malloc(sizeof(double) * (npts > 0 ? npts : 1));
    double *tr = (double*)malloc(sizeof(double) * (ms > 0 ? ms : 1));
    for (int64_t i = 0; i < npts; ++i) td[i] = b[o.pidx[i]];   /* s = Aᵀb */
    memcpy(tr, b + npts, sizeof(double) * ms);
    op_adj(&o, td, tr, s);
    /* z = M⁻¹ s per block (full ids); columns outside every block: z = s; removed columns: 0 */
#define APPLY_M()                                                                                   \
    do {                                                                                            \
        memcpy(z, s, sizeof(double) * nf);                                                          \
        _Pragma("omp parallel for schedule(static)") for (int64_t bb = 0; bb < nblk; ++bb) {       \
            const int64_t b0 = bptr[bb];                                                            \
            const int k = (int)(bptr[bb + 1] - b0);                                                 \
            const double* Rb = R + bb * KB * KB;                                                    \
            double w[KB];                                                                           \
            for (int j = 0; j < k; ++j) { /* Rᵀ w = s_b */                                         \
                double a = s[fcol[b0 + j]];                                                         \
                for (int l = 0; l < j; ++l) a -= Rb[l * KB + j] * w[l];                             \
                w[j] = Rb[j * KB + j] > 0.0 ? a / Rb[j * KB + j] : 0.0;                             \
            }                                                                                       \
            for (int j = k - 1; j >= 0; --j) { /* R z_b = w */                                     \
                double a = w[j];                                                                    \
                for (int l = j + 1; l < k; ++l) a -= Rb[j * KB + l] * w[l];                         \
                w[j] = Rb[j * KB + j] > 0.0 ? a / Rb[j * KB + j] : 0.0;                             \
            }                                                                                       \
            for (int j = 0; j < k; ++j) z[fcol[b0 + j]] = w[j];                                     \
        }                                                                                           \
    } while (0)
    APPLY_M();
    memcpy(p, z, sizeof(double) * nf);
    double rho = dot(nf, s, z);
    const double t1 = omp_get_wtime();
    if (maxit <= 0) maxit = 4 * n;
    int64_t it = 0;
    double snorm = sqrt(dot(nf, s, s)), rnorm = sqrt(dot(m, b, b));
    for (; fixed_iters > 0 ? it < fixed_iters : it < maxit; ++it) {
        if (fixed_iters <= 0 && snorm <= atol * anorm_f * rnorm) break;
        op_fwd(&o, p, td, tr);
        const double gam = dot(npts, td, td) + dot(ms, tr, tr);
        if (!(gam > 0.0)) break;
        const double alpha = rho / gam;
#pragma omp parallel for schedule(static)
        for (int64_t j = 0; j < nf; ++j) xf[j] += alpha * p[j];
        op_adj(&o, td, tr, q);
#pragma omp parallel for schedule(static)
        for (int64_t j = 0; j < nf; ++j) s[j] -= alpha * q[j];
        APPLY_M();
        const double rho2 = dot(nf, s, z);
        const double beta = rho2 / rho;
        rho = rho2;
#pragma omp parallel for schedule(static)
        for (int64_t j = 0; j < nf; ++j) p[j] = z[j] + beta * p[j];
        if (fixed_iters <= 0) {   /* the stopping test's ‖s‖ and ‖b − Ax‖ */
            snorm = sqrt(dot(nf, s, s));
            op_fwd(&o, xf, td, tr);
            double r2 = 0.0;
#pragma omp parallel for reduction(+ : r2) schedule(static)
            for (int64_t i = 0; i < npts; ++i) r2 += (b[o.pidx[i]] - td[i]) * (b[o.pidx[i]] - td[i]);
#pragma omp parallel for reduction(+ : r2) schedule(static)
            for (int64_t i = 0; i < ms; ++i) r2 += (b[npts + i] - tr[i]) * (b[npts + i] - tr[i]);
            rnorm = sqrt(r2);
        }
    }
#undef APPLY_M
    const double t2 = omp_get_wtime();
    for (int64_t j = 0; j < n; ++j) x[j] = xf[keep[j]];
    stats[0] = (double)it;
    stats[1] = t2 - t1;
    stats[2] = t1 - t0;
    stats[3] = (double)omp_get_max_threads();
    stats[4] = snorm;
    stats[5] = rnorm;
    stats[6] = anorm_f;
    free(R); free(fcol); free(s); free(z); free(p); free(q); free(xf); free(td); free(tr);
    op_free(&o);
    return 0;
}
