// build.hip — device formation of the least-squares operator (replaces the scipy assembly of
// LSsurf/smooth_fit.py:613-627 and lin_op.toCSR, lin_op.py:745-753).
//
//   COO (r, c, v) ──drop v==0, Ip_c──▶ row buckets ──sort (col, input order), sum duplicates,
//   drop zero sums──▶ canonical CSR G ──▶ transpose GT ──▶ SELL-64 copies A, AT with values
//   diag(rs)·G·diag(cs).
//
// Everything is integer bookkeeping plus one f64 add per duplicate, so the formed G is
// bit-identical to scipy's for any input whose duplicates are at most pairs (the smooth_fit
// systems have none); see DESIGN.md §Formation.
#include <algorithm>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "system.hpp"

namespace lsq {

namespace {

constexpr int64_t MAX_SEG = 1 << 16;   // longest row / column handled by the per-segment sort

struct BuildErr {
    unsigned long long count;
    long long first;      // first offending COO index
    int kind;             // 1 row out of range, 2 col out of range, 3 segment too long
};

__global__ __launch_bounds__(BLOCK) void k_coo_count(int64_t nnz, int64_t m, int64_t n_full,
                                                     const int64_t* __restrict__ r,
                                                     const int64_t* __restrict__ c,
                                                     const double* __restrict__ v,
                                                     const int32_t* __restrict__ colmap,
                                                     unsigned long long* __restrict__ cnt,
                                                     BuildErr* err) {
    for (int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * BLOCK) {
        if (v[e] == 0.0) continue;                      // lin_op.toCSR: good = v != 0
        const int64_t ri = r[e], cj = c[e];
        int kind = 0;
        if (ri < 0 || ri >= m) kind = 1;
        else if (cj < 0 || cj >= n_full) kind = 2;
        if (kind) {
            if (atomicAdd(&err->count, 1ull) == 0) { err->first = e; err->kind = kind; }
            continue;
        }
        if (colmap && colmap[cj] < 0) continue;         // column removed by Ip_c
        atomicAdd(&cnt[ri], 1ull);
    }
}

__global__ __launch_bounds__(BLOCK) void k_coo_scatter(int64_t nnz, const int64_t* __restrict__ r,
                                                       const int64_t* __restrict__ c,
                                                       const double* __restrict__ v,
                                                       const int32_t* __restrict__ colmap,
                                                       const int64_t* __restrict__ off,
                                                       unsigned long long* __restrict__ cur,
                                                       int32_t* __restrict__ tc, double* __restrict__ tv,
                                                       int64_t* __restrict__ te) {
    for (int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * BLOCK) {
        const double ve = v[e];
        if (ve == 0.0) continue;
        const int64_t ri = r[e];
        int64_t cj = c[e];
        if (colmap) {
            cj = colmap[cj];
            if (cj < 0) continue;
        }
        const int64_t pos = off[ri] + (int64_t)atomicAdd(&cur[ri], 1ull);
        tc[pos] = (int32_t)cj;
        tv[pos] = ve;
        te[pos] = e;
    }
}

// One thread per row: insertion sort by (col, input index), then sum duplicates in input
// order and drop zero sums; the deduplicated entries are written to the segment's front.
__global__ __launch_bounds__(BLOCK) void k_row_sort_dedupe(int64_t m, const int64_t* __restrict__ off,
                                                           int32_t* __restrict__ tc, double* __restrict__ tv,
                                                           int64_t* __restrict__ te,
                                                           int64_t* __restrict__ dcnt, BuildErr* err) {
    for (int64_t row = (int64_t)blockIdx.x * BLOCK + threadIdx.x; row < m; row += (int64_t)gridDim.x * BLOCK) {
        const int64_t b = off[row], L = off[row + 1] - b;
        if (L > MAX_SEG) {
            if (atomicAdd(&err->count, 1ull) == 0) { err->first = row; err->kind = 3; }
            dcnt[row] = 0;
            continue;
        }
        for (int64_t i = 1; i < L; ++i) {
            const int32_t kc = tc[b + i];
            const double kv = tv[b + i];
            const int64_t ke = te[b + i];
            int64_t j = i - 1;
            while (j >= 0 && (tc[b + j] > kc || (tc[b + j] == kc && te[b + j] > ke))) {
                tc[b + j + 1] = tc[b + j];
                tv[b + j + 1] = tv[b + j];
                te[b + j + 1] = te[b + j];
                --j;
            }
            tc[b + j + 1] = kc;
            tv[b + j + 1] = kv;
            te[b + j + 1] = ke;
        }
        int64_t out = 0;
        int64_t i = 0;
        while (i < L) {
            const int32_t col = tc[b + i];
            double s = tv[b + i];
            int64_t k = i + 1;
            while (k < L && tc[b + k] == col) { s += tv[b + k]; ++k; }
            if (s != 0.0) {                     // scipy csr_matmat drops zero sums
                tc[b + out] = col;
                tv[b + out] = s;
                ++out;
            }
            i = k;
        }
        dcnt[row] = out;
    }
}

__global__ __launch_bounds__(BLOCK) void k_compact(int64_t m, const int64_t* __restrict__ off,
                                                   const int32_t* __restrict__ tc, const double* __restrict__ tv,
                                                   const int64_t* __restrict__ rp, int32_t* __restrict__ ci,
                                                   double* __restrict__ val) {
    for (int64_t row = (int64_t)blockIdx.x * BLOCK + threadIdx.x; row < m; row += (int64_t)gridDim.x * BLOCK) {
        const int64_t b = off[row], o = rp[row], L = rp[row + 1] - o;
        for (int64_t k = 0; k < L; ++k) {
            ci[o + k] = tc[b + k];
            val[o + k] = tv[b + k];
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_u64_to_i64(int64_t n, const unsigned long long* __restrict__ a,
                                                      int64_t* __restrict__ b) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK)
        b[i] = (int64_t)a[i];
}

// ---- transpose -------------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_col_count(int64_t m, const int64_t* __restrict__ rp,
                                                     const int32_t* __restrict__ ci,
                                                     unsigned long long* __restrict__ cnt) {
    for (int64_t row = (int64_t)blockIdx.x * BLOCK + threadIdx.x; row < m; row += (int64_t)gridDim.x * BLOCK)
        for (int64_t e = rp[row]; e < rp[row + 1]; ++e) atomicAdd(&cnt[ci[e]], 1ull);
}

__global__ __launch_bounds__(BLOCK) void k_t_scatter(int64_t m, const int64_t* __restrict__ rp,
                                                     const int32_t* __restrict__ ci, const double* __restrict__ val,
                                                     const int64_t* __restrict__ trp,
                                                     unsigned long long* __restrict__ cur,
                                                     int32_t* __restrict__ tci, double* __restrict__ tval) {
    for (int64_t row = (int64_t)blockIdx.x * BLOCK + threadIdx.x; row < m; row += (int64_t)gridDim.x * BLOCK)
        for (int64_t e = rp[row]; e < rp[row + 1]; ++e) {
            const int32_t j = ci[e];
            const int64_t pos = trp[j] + (int64_t)atomicAdd(&cur[j], 1ull);
            tci[pos] = (int32_t)row;
            tval[pos] = val[e];
        }
}

// Column segments: sort by row index (unique within a column) -> deterministic GT.
__global__ __launch_bounds__(BLOCK) void k_seg_sort(int64_t n, const int64_t* __restrict__ rp,
                                                    int32_t* __restrict__ ci, double* __restrict__ val,
                                                    BuildErr* err) {
    for (int64_t row = (int64_t)blockIdx.x * BLOCK + threadIdx.x; row < n; row += (int64_t)gridDim.x * BLOCK) {
        const int64_t b = rp[row], L = rp[row + 1] - b;
        if (L > MAX_SEG) {
            if (atomicAdd(&err->count, 1ull) == 0) { err->first = row; err->kind = 3; }
            continue;
        }
        for (int64_t i = 1; i < L; ++i) {
            const int32_t kc = ci[b + i];
            const double kv = val[b + i];
            int64_t j = i - 1;
            while (j >= 0 && ci[b + j] > kc) {
                ci[b + j + 1] = ci[b + j];
                val[b + j + 1] = val[b + j];
                --j;
            }
            ci[b + j + 1] = kc;
            val[b + j + 1] = kv;
        }
    }
}

// ---- SELL-64 ---------------------------------------------------------------------------------
// SELL row r holds CSR row perm[r] (perm may be null = identity); column ids may be remapped
// through cmap (AT: A's CSR row ids -> A's SELL row ids).
__global__ __launch_bounds__(BLOCK) void k_slice_width(int64_t rows, int64_t nslices,
                                                       const int64_t* __restrict__ rp,
                                                       const int32_t* __restrict__ perm,
                                                       int64_t* __restrict__ wid) {
    for (int64_t s = (int64_t)blockIdx.x * BLOCK + threadIdx.x; s < nslices; s += (int64_t)gridDim.x * BLOCK) {
        int64_t w = 0;
        const int64_t r0 = s * SELL_C;
        const int64_t r1 = r0 + SELL_C < rows ? r0 + SELL_C : rows;
        for (int64_t r = r0; r < r1; ++r) {
            const int64_t q = perm ? perm[r] : r;
            if (q >= 0) w = max(w, rp[q + 1] - rp[q]);
        }
        wid[s] = w * SELL_C;
    }
}

__global__ __launch_bounds__(BLOCK) void k_sell_cols(int64_t rows, const int64_t* __restrict__ rp,
                                                     const int32_t* __restrict__ ci,
                                                     const int32_t* __restrict__ perm,
                                                     const int32_t* __restrict__ cmap,
                                                     const int64_t* __restrict__ sp, int32_t* __restrict__ sci) {
    for (int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < rows; r += (int64_t)gridDim.x * BLOCK) {
        const int64_t s = r / SELL_C, lane = r % SELL_C;
        const int64_t q = perm ? perm[r] : r;   // q < 0: empty row
        const int64_t base = sp[s], W = (sp[s + 1] - base) / SELL_C;
        const int64_t b = q >= 0 ? rp[q] : 0, L = q >= 0 ? rp[q + 1] - b : 0;
        for (int64_t k = 0; k < W; ++k) {
            int32_t c = L ? ci[b + (k < L ? k : L - 1)] : 0;
            sci[base + k * SELL_C + lane] = cmap && L ? cmap[c] : c;
        }
    }
}

// Row order of A's SELL copy.  Rows are grouped by length (equal-length rows share slices: no
// padding).  Within a length, the first `n_sorted` rows (the data rows: they arrive in point
// order, which is random in space) are ordered by their first column, so the rows of a slice
// gather from a few cache lines; the other rows (stencil rows, already in grid order) keep their
// order, so each stencil part stays contiguous and Aᵀ's gathers of u stay coalesced.
__global__ __launch_bounds__(BLOCK) void k_row_keys(int64_t m, int64_t n_sorted, const int64_t* __restrict__ rp,
                                                    const int32_t* __restrict__ ci,
                                                    unsigned long long* __restrict__ key,
                                                    int32_t* __restrict__ id) {
    for (int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < m; r += (int64_t)gridDim.x * BLOCK) {
        const int64_t L = rp[r + 1] - rp[r];
        const bool by_col = r < n_sorted && L > 0;
        const unsigned long long v = by_col ? (unsigned long long)(uint32_t)ci[rp[r]] : (unsigned long long)r;
        key[r] = ((unsigned long long)L << 33) | ((unsigned long long)(by_col ? 0 : 1) << 32) | v;
        id[r] = (int32_t)r;
    }
}

__global__ __launch_bounds__(BLOCK) void k_keep_list(int64_t n_full, const int32_t* __restrict__ colmap,
                                                     int32_t* __restrict__ keep) {
    for (int64_t f = (int64_t)blockIdx.x * BLOCK + threadIdx.x; f < n_full; f += (int64_t)gridDim.x * BLOCK) {
        const int32_t c = colmap ? colmap[f] : (int32_t)f;
        if (c >= 0) keep[c] = (int32_t)f;
    }
}

__global__ __launch_bounds__(BLOCK) void k_scatter_cs(int64_t n, const int32_t* __restrict__ keep,
                                                      const double* __restrict__ cs, double* __restrict__ csf) {
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK)
        csf[keep[j]] = cs[j];
}

// per stencil part: min and max of the row scale over its rows; blockIdx = (part, chunk of
// MINMAX_CHUNKS), one (min, max) pair per block, combined on the host
constexpr int MINMAX_CHUNKS = 64;
__global__ __launch_bounds__(BLOCK) void k_part_minmax(const MfDesc* __restrict__ d, const double* __restrict__ rs,
                                                       double* __restrict__ out) {
    __shared__ double lo[BLOCK], hi[BLOCK];
    const int p = blockIdx.x / MINMAX_CHUNKS, chunk = blockIdx.x % MINMAX_CHUNKS;
    const MfPart& P = d->p[p];
    double a = INFINITY, b = -INFINITY;
    for (int64_t r = (int64_t)chunk * BLOCK + threadIdx.x; r < P.n_eq; r += (int64_t)MINMAX_CHUNKS * BLOCK) {
        const double x = rs[P.row0 + r];
        a = fmin(a, x);
        b = fmax(b, x);
    }
    lo[threadIdx.x] = a;
    hi[threadIdx.x] = b;
    __syncthreads();
    for (int k = BLOCK / 2; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) {
            lo[threadIdx.x] = fmin(lo[threadIdx.x], lo[threadIdx.x + k]);
            hi[threadIdx.x] = fmax(hi[threadIdx.x], hi[threadIdx.x + k]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = lo[0];
        out[2 * blockIdx.x + 1] = hi[0];
    }
}

// position -> GdT row (compact column) of the node enumeration, -1 for padding / removed columns
__global__ __launch_bounds__(BLOCK) void k_enum_perm(const MfDesc* __restrict__ d, int64_t ne,
                                                     const int32_t* __restrict__ colmap, int32_t* __restrict__ perm) {
    for (int64_t pos = (int64_t)blockIdx.x * BLOCK + threadIdx.x; pos < ne; pos += (int64_t)gridDim.x * BLOCK) {
        int32_t q = -1;
        for (int g = 0; g < d->n_grids; ++g) {
            const MfGrid& G = d->g[g];
            if (G.nparts && pos >= G.node0 && pos < (int64_t)G.node0 + G.nodes) {
                const int64_t f = G.col0 + (pos - G.node0);
                q = colmap ? colmap[f] : (int32_t)f;
            }
        }
        perm[pos] = q;
    }
}

__global__ __launch_bounds__(BLOCK) void k_invert(int64_t m, const int32_t* __restrict__ perm,
                                                  int32_t* __restrict__ inv) {
    for (int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < m; r += (int64_t)gridDim.x * BLOCK)
        inv[perm[r]] = (int32_t)r;
}

// val_sell = (g * rs[row]) * cs[col]; `rowsc`/`colsc` index by the CSR's own row / column ids.
__global__ __launch_bounds__(BLOCK) void k_sell_vals(int64_t rows, const int64_t* __restrict__ rp,
                                                     const int32_t* __restrict__ ci, const double* __restrict__ g,
                                                     const double* __restrict__ rowsc,
                                                     const double* __restrict__ colsc, int transposed,
                                                     const int32_t* __restrict__ perm,
                                                     const int64_t* __restrict__ sp, double* __restrict__ sval) {
    for (int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < rows; r += (int64_t)gridDim.x * BLOCK) {
        const int64_t s = r / SELL_C, lane = r % SELL_C;
        const int64_t q = perm ? perm[r] : r;   // CSR row (< 0: empty row)
        const int64_t base = sp[s], W = (sp[s + 1] - base) / SELL_C;
        const int64_t b = q >= 0 ? rp[q] : 0, L = q >= 0 ? rp[q + 1] - b : 0;
        for (int64_t k = 0; k < W; ++k) {
            double x = 0.0;
            if (k < L) {
                const int32_t c = ci[b + k];
                // A: row scale of q, col scale of c.  AT: row scale of c, col scale of q.
                // colsc == nullptr: no column factor (the stencil operator applies cs itself)
                if (transposed)
                    x = colsc ? (g[b + k] * rowsc[c]) * colsc[q] : g[b + k] * rowsc[c];
                else
                    x = colsc ? (g[b + k] * rowsc[q]) * colsc[c] : g[b + k] * rowsc[q];
            }
            sval[base + k * SELL_C + lane] = x;
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_rowscale(int64_t m, const double* __restrict__ w,
                                                    const uint8_t* __restrict__ keep, double* __restrict__ rs) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += (int64_t)gridDim.x * BLOCK)
        rs[i] = keep[i] ? w[i] : 0.0;
}

// Jacobi column scaling: cs_j = 1/||(diag(rs) G)_{:,j}||  (1 for an empty column).
// raw = 1 stores the squared norm (distributed: summed across ranks before finishing).
__global__ __launch_bounds__(BLOCK) void k_colnorm(int64_t n, const int64_t* __restrict__ trp,
                                                   const int32_t* __restrict__ tci, const double* __restrict__ tval,
                                                   const double* __restrict__ rs, double* __restrict__ cs, int raw) {
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK) {
        double s = 0.0;
        for (int64_t e = trp[j]; e < trp[j + 1]; ++e) {
            const double a = tval[e] * rs[tci[e]];
            s += a * a;
        }
        cs[j] = raw ? s : (s > 0.0 ? 1.0 / sqrt(s) : 1.0);
    }
}

__global__ __launch_bounds__(BLOCK) void k_cs_finish(int64_t n, double* __restrict__ cs) {
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK) {
        const double s = cs[j];
        cs[j] = s > 0.0 ? 1.0 / sqrt(s) : 1.0;
    }
}

__global__ __launch_bounds__(BLOCK) void k_mask01(int64_t n, uint8_t* __restrict__ k) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) k[i] = k[i] ? 1 : 0;
}

__global__ __launch_bounds__(BLOCK) void k_fill(int64_t n, double v, double* __restrict__ a) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) a[i] = v;
}

__global__ __launch_bounds__(BLOCK) void k_csr_spmv(int64_t rows, const int64_t* __restrict__ rp,
                                                    const int32_t* __restrict__ ci, const double* __restrict__ val,
                                                    const double* __restrict__ x, double* __restrict__ y) {
    for (int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < rows; r += (int64_t)gridDim.x * BLOCK) {
        double acc = 0.0;
        for (int64_t e = rp[r]; e < rp[r + 1]; ++e) acc += val[e] * x[ci[e]];
        y[r] = acc;
    }
}

// per-block partials of Σ (w_i u_i)² and Σ u_i² over rows [first, first + count), u = G x (the
// row products in k_csr_spmv's order), w = the row weights (smooth_fit.py:324-331: R and RMS of
// each constraint type)
__global__ __launch_bounds__(BLOCK) void k_rows_sumsq(int64_t first, int64_t count, const int64_t* __restrict__ rp,
                                                      const int32_t* __restrict__ ci, const double* __restrict__ val,
                                                      const double* __restrict__ x, const double* __restrict__ w,
                                                      double* __restrict__ pw, double* __restrict__ pu) {
    double aw = 0.0, au = 0.0;
    for (int64_t r = first + (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < first + count; r += (int64_t)gridDim.x * BLOCK) {
        double acc = 0.0;
        for (int64_t e = rp[r]; e < rp[r + 1]; ++e) acc += val[e] * x[ci[e]];
        const double rc = (w ? w[r] : 1.0) * acc;
        aw += rc * rc;
        au += acc * acc;
    }
    __shared__ double red[4];
    const double sw = block_sum(aw, red);
    __syncthreads();
    const double su = block_sum(au, red);
    if (threadIdx.x == 0) {
        pw[blockIdx.x] = sw;
        pu[blockIdx.x] = su;
    }
}

// Row r of stencil part P (r − P.row0 = k, the centre's position in the part's box), straight from
// the part descriptor as k_gen_rows generates it: entry t at full column col0 + ravel(c + off_t),
// value val_t (· F[fsel_t][k] for a field-valued part).  xf: full column space (removed columns 0).
__device__ double mf_stencil_row(const MfDesc& d, const MfPart& P, int64_t k, const double* __restrict__ xf) {
    const MfGrid& G = d.g[P.grid];
    const int nd = G.ndim;
    int64_t sub[3] = {0, 0, 0}, gst[3] = {1, 1, 1}, rem = k;
    for (int e = nd - 1; e >= 0; --e) {
        const int64_t ext = P.hi[e] - P.lo[e];
        sub[e] = P.lo[e] + rem % ext;
        rem /= ext;
        if (e < nd - 1) gst[e] = gst[e + 1] * G.shape[e + 1];
    }
    double acc = 0.0;
    for (int t = 0; t < P.ntpl; ++t) {
        int64_t col = G.col0;
        for (int e = 0; e < nd; ++e) col += (sub[e] + P.off[t][e]) * gst[e];
        const double v = P.var ? P.val[t] * P.F[(int64_t)P.fsel[t] * P.n_eq + k] : P.val[t];
        acc += v * xf[col];
    }
    return acc;
}

// k_rows_sumsq for rows of the stencil parts of a lazily formed system (rows ≥ npts)
__global__ __launch_bounds__(BLOCK) void k_rows_sumsq_mf(const MfDesc* __restrict__ dd, int64_t first, int64_t count,
                                                         const double* __restrict__ xf, const double* __restrict__ w,
                                                         double* __restrict__ pw, double* __restrict__ pu) {
    const MfDesc& d = *dd;
    double aw = 0.0, au = 0.0;
    for (int64_t r = first + (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < first + count; r += (int64_t)gridDim.x * BLOCK) {
        int p = 0;
        while (p + 1 < d.n_parts && r >= d.p[p + 1].row0) ++p;
        const MfPart& P = d.p[p];
        const double acc = mf_stencil_row(d, P, r - P.row0, xf);
        const double rc = (w ? w[r] : 1.0) * acc;
        aw += rc * rc;
        au += acc * acc;
    }
    __shared__ double red[4];
    const double sw = block_sum(aw, red);
    __syncthreads();
    const double su = block_sum(au, red);
    if (threadIdx.x == 0) {
        pw[blockIdx.x] = sw;
        pu[blockIdx.x] = su;
    }
}

// distributed layout: mark referenced columns; relabel columns to local ids and re-sort rows
__global__ __launch_bounds__(BLOCK) void k_flag_cols(int64_t nnz, const int32_t* __restrict__ ci,
                                                     uint8_t* __restrict__ flags) {
    for (int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * BLOCK)
        flags[ci[e]] = 1;
}

__global__ __launch_bounds__(BLOCK) void k_relabel_rows(int64_t m, const int64_t* __restrict__ rp,
                                                        int32_t* __restrict__ ci, double* __restrict__ val,
                                                        const int32_t* __restrict__ map,
                                                        unsigned long long* __restrict__ bad) {
    for (int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < m; r += (int64_t)gridDim.x * BLOCK) {
        const int64_t b = rp[r], L = rp[r + 1] - b;
        for (int64_t k = 0; k < L; ++k) {
            const int32_t c = map[ci[b + k]];
            if (c < 0) atomicAdd(bad, 1ull);
            ci[b + k] = c;
        }
        for (int64_t i = 1; i < L; ++i) {
            const int32_t kc = ci[b + i];
            const double kv = val[b + i];
            int64_t j = i - 1;
            while (j >= 0 && ci[b + j] > kc) {
                ci[b + j + 1] = ci[b + j];
                val[b + j + 1] = val[b + j];
                --j;
            }
            ci[b + j + 1] = kc;
            val[b + j + 1] = kv;
        }
    }
}

void check_err(BuildErr* d_err, hipStream_t s, const char* stage) {
    BuildErr h{};
    HIP_CHECK(hipMemcpyAsync(&h, d_err, sizeof(BuildErr), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (h.count) {
        const char* what = h.kind == 1 ? "row index out of range" : h.kind == 2 ? "column index out of range"
                                                                                : "segment longer than 65536 entries";
        throw std::invalid_argument(std::string(stage) + ": " + what + " (first at " + std::to_string(h.first) +
                                    ", " + std::to_string(h.count) + " total)");
    }
}

// SELL copy of `rows` rows: SELL row r = CSR row perm[r] of C (S.perm; identity if empty; < 0
// = empty row); column ids optionally mapped through cmap.
void build_sell(Sell& S, const Csr& C, int64_t rows, const int32_t* cmap, hipStream_t st) {
    S.rows = rows;
    S.nslices = (rows + SELL_C - 1) / SELL_C;
    S.sp.alloc(S.nslices + 1);
    S.sp.zero(st);
    const int32_t* perm = S.perm.n ? S.perm.p : nullptr;
    hipLaunchKernelGGL(k_slice_width, dim3(grid_for(S.nslices)), dim3(BLOCK), 0, st, rows, S.nslices, C.rp.p, perm,
                       S.sp.p);
    KERNEL_CHECK();
    S.nent = exclusive_scan_i64(S.sp.p, S.nslices + 1, st);
    S.ci.alloc(std::max<int64_t>(S.nent, 1));
    S.val.alloc(std::max<int64_t>(S.nent, 1));
    // lanes past the last row of the final slice are never written by k_sell_cols/k_sell_vals:
    // give them column 0 and value 0 so any read of them is in bounds and contributes nothing
    S.ci.zero(st);
    S.val.zero(st);
    hipLaunchKernelGGL(k_sell_cols, dim3(grid_for(rows)), dim3(BLOCK), 0, st, rows, C.rp.p, C.ci.p, perm, cmap, S.sp.p,
                       S.ci.p);
    KERNEL_CHECK();
}

// A's SELL row order (k_row_keys): one radix sort of 64-bit keys.
void locality_order(const Csr& G, int64_t m, int64_t n_sorted, DBuf<int32_t>& perm, DBuf<int32_t>& inv,
                    hipStream_t st) {
    perm.alloc(std::max<int64_t>(m, 1));
    inv.alloc(std::max<int64_t>(m, 1));
    if (m == 0) return;
    if (m >= (int64_t(1) << 31)) throw std::invalid_argument("more than 2^31 rows");
    DBuf<unsigned long long> k0(m), k1(m);
    DBuf<int32_t> id(m);
    hipLaunchKernelGGL(k_row_keys, dim3(grid_for(m)), dim3(BLOCK), 0, st, m, n_sorted, G.rp.p, G.ci.p, k0.p, id.p);
    KERNEL_CHECK();
    size_t tmp_bytes = 0;
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k0.p, k1.p, id.p, perm.p, (int)m, 0, 64, st));
    DBuf<unsigned char> tmp((int64_t)tmp_bytes + 1);
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tmp_bytes, k0.p, k1.p, id.p, perm.p, (int)m, 0, 64, st));
    hipLaunchKernelGGL(k_invert, dim3(grid_for(m)), dim3(BLOCK), 0, st, m, perm.p, inv.p);
    KERNEL_CHECK();
    HIP_CHECK(hipStreamSynchronize(st));
}

}  // namespace

void form_from_coo(System& S, int64_t m, int64_t n_full, int64_t nnz, const int64_t* r, const int64_t* c,
                   const double* v) {
    hipStream_t st = S.stream;
    const int64_t n = S.have_colmap ? S.n_keep : n_full;   // compact width (lsq_set_col_map)
    DBuf<int64_t> dr(nnz), dc(nnz);
    DBuf<double> dv(nnz);
    dr.upload(r, nnz, st);
    dc.upload(c, nnz, st);
    dv.upload(v, nnz, st);
    DBuf<BuildErr> err(1);
    err.zero(st);
    DBuf<unsigned long long> cnt(m + 1), cur(m + 1);
    cnt.zero(st);
    cur.zero(st);
    const int32_t* cmap = S.have_colmap ? S.colmap.p : nullptr;
    const int gE = grid_for(nnz);
    hipLaunchKernelGGL(k_coo_count, dim3(gE), dim3(BLOCK), 0, st, nnz, m, n_full, dr.p, dc.p, dv.p, cmap, cnt.p, err.p);
    KERNEL_CHECK();
    check_err(err.p, st, "lsq_set_matrix_coo");
    DBuf<int64_t> off(m + 1);
    hipLaunchKernelGGL(k_u64_to_i64, dim3(grid_for(m + 1)), dim3(BLOCK), 0, st, m + 1, cnt.p, off.p);
    KERNEL_CHECK();
    const int64_t kept = exclusive_scan_i64(off.p, m + 1, st);
    DBuf<int32_t> tc(std::max<int64_t>(kept, 1));
    DBuf<double> tv(std::max<int64_t>(kept, 1));
    DBuf<int64_t> te(std::max<int64_t>(kept, 1));
    hipLaunchKernelGGL(k_coo_scatter, dim3(gE), dim3(BLOCK), 0, st, nnz, dr.p, dc.p, dv.p, cmap, off.p, cur.p, tc.p,
                       tv.p, te.p);
    KERNEL_CHECK();
    dr.release();
    dc.release();
    dv.release();
    DBuf<int64_t> dcnt(m + 1);
    dcnt.zero(st);
    hipLaunchKernelGGL(k_row_sort_dedupe, dim3(grid_for(m)), dim3(BLOCK), 0, st, m, off.p, tc.p, tv.p, te.p, dcnt.p,
                       err.p);
    KERNEL_CHECK();
    check_err(err.p, st, "lsq_set_matrix_coo");
    te.release();

    Csr& G = S.G;
    G.m = m;
    G.n = n;
    G.rp = std::move(dcnt);
    G.nnz = exclusive_scan_i64(G.rp.p, m + 1, st);
    G.ci.alloc(std::max<int64_t>(G.nnz, 1));
    G.val.alloc(std::max<int64_t>(G.nnz, 1));
    hipLaunchKernelGGL(k_compact, dim3(grid_for(m)), dim3(BLOCK), 0, st, m, off.p, tc.p, tv.p, G.rp.p, G.ci.p, G.val.p);
    KERNEL_CHECK();
    tc.release();
    tv.release();
    off.release();
    S.n_sorted_rows = 0;
    S.mf = false;   // generic operator: assembled SELL only
    finish_formation(S);
}

// G (canonical CSR, set) -> GT, SELL copies, default scaling state.
namespace {

// CSR transpose of the first `rows` rows of G (entries of a column in ascending row order).
void transpose_rows(const Csr& G, int64_t rows, Csr& T, hipStream_t st) {
    const int64_t n = G.n;
    DBuf<BuildErr> err(1);
    err.zero(st);
    T.m = n;
    T.n = rows;
    DBuf<unsigned long long> ccnt(n + 1), ccur(n + 1);
    ccnt.zero(st);
    ccur.zero(st);
    hipLaunchKernelGGL(k_col_count, dim3(grid_for(rows)), dim3(BLOCK), 0, st, rows, G.rp.p, G.ci.p, ccnt.p);
    KERNEL_CHECK();
    T.rp.alloc(n + 1);
    hipLaunchKernelGGL(k_u64_to_i64, dim3(grid_for(n + 1)), dim3(BLOCK), 0, st, n + 1, ccnt.p, T.rp.p);
    KERNEL_CHECK();
    T.nnz = exclusive_scan_i64(T.rp.p, n + 1, st);
    T.ci.alloc(std::max<int64_t>(T.nnz, 1));
    T.val.alloc(std::max<int64_t>(T.nnz, 1));
    hipLaunchKernelGGL(k_t_scatter, dim3(grid_for(rows)), dim3(BLOCK), 0, st, rows, G.rp.p, G.ci.p, G.val.p, T.rp.p,
                       ccur.p, T.ci.p, T.val.p);
    KERNEL_CHECK();
    hipLaunchKernelGGL(k_seg_sort, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, T.rp.p, T.ci.p, T.val.p, err.p);
    KERNEL_CHECK();
    check_err(err.p, st, "matrix transpose");
}

}  // namespace

// Assembled SELL copies of the whole operator (A rows grouped by length, data rows by first
// column; AT's column ids = A's SELL row ids).
void ensure_sell(System& S) {
    if (S.sell_built) return;
    ensure_full_csr(S);
    hipStream_t st = S.stream;
    DBuf<int32_t> inv;
    locality_order(S.G, S.G.m, S.n_sorted_rows, S.A.perm, inv, st);
    build_sell(S.A, S.G, S.G.m, nullptr, st);
    build_sell(S.AT, S.GT, S.GT.m, inv.p, st);
    HIP_CHECK(hipStreamSynchronize(st));
    S.sell_built = true;
    S.cs_mode = -1;   // values are filled by the next refresh
    S.iter_ready = false;
}

namespace {

__global__ __launch_bounds__(BLOCK) void k_c32_count(int64_t rows, const int32_t* __restrict__ perm,
                                                     const int64_t* __restrict__ srp, int64_t* __restrict__ cnt) {
    for (int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < rows; r += (int64_t)gridDim.x * BLOCK) {
        const int32_t q = perm[r];
        cnt[r] = q >= 0 ? srp[q + 1] - srp[q] : 0;
    }
}

__global__ __launch_bounds__(BLOCK) void k_c32_fill(int64_t rows, const int32_t* __restrict__ perm,
                                                    const int64_t* __restrict__ srp, const int32_t* __restrict__ sci,
                                                    const int32_t* __restrict__ cmap, const int64_t* __restrict__ off,
                                                    int32_t* __restrict__ rp, int32_t* __restrict__ ci) {
    for (int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x; r <= rows; r += (int64_t)gridDim.x * BLOCK) {
        rp[r] = (int32_t)off[r];
        if (r == rows) continue;
        const int32_t q = perm[r];
        if (q < 0) continue;
        for (int64_t e = srp[q], o = off[r]; e < srp[q + 1]; ++e, ++o) ci[o] = cmap ? cmap[sci[e]] : sci[e];
    }
}

// values: transposed source, row scale by the source column (= the original row of A)
__global__ __launch_bounds__(BLOCK) void k_c32_vals(int64_t rows, const int32_t* __restrict__ perm,
                                                    const int64_t* __restrict__ srp, const int32_t* __restrict__ sci,
                                                    const double* __restrict__ sval, const double* __restrict__ rs,
                                                    const int32_t* __restrict__ rp, double* __restrict__ val) {
    for (int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < rows; r += (int64_t)gridDim.x * BLOCK) {
        const int32_t q = perm[r];
        if (q < 0) continue;
        for (int64_t e = srp[q], o = rp[r]; e < srp[q + 1]; ++e, ++o) val[o] = sval[e] * rs[sci[e]];
    }
}

void build_csr32(Csr32& C, const Csr& src, int64_t rows, const int32_t* cmap, hipStream_t st) {
    C.rows = rows;
    DBuf<int64_t> off(rows + 1);
    off.zero(st);
    hipLaunchKernelGGL(k_c32_count, dim3(grid_for(rows)), dim3(BLOCK), 0, st, rows, C.perm.p, src.rp.p, off.p);
    KERNEL_CHECK();
    C.nnz = exclusive_scan_i64(off.p, rows + 1, st);
    if (C.nnz >= (int64_t(1) << 31)) throw std::invalid_argument("data part too large for 32-bit offsets");
    C.rp.alloc(rows + 1);
    C.ci.alloc(std::max<int64_t>(C.nnz, 1));
    C.val.alloc(std::max<int64_t>(C.nnz, 1));
    hipLaunchKernelGGL(k_c32_fill, dim3(grid_for(rows + 1)), dim3(BLOCK), 0, st, rows, C.perm.p, src.rp.p, src.ci.p,
                       cmap, off.p, C.rp.p, C.ci.p);
    KERNEL_CHECK();
    HIP_CHECK(hipStreamSynchronize(st));
}

// Data rows of a structured system: Ad (SELL rows = data rows by first column, full column ids)
// and ATd (SELL rows = node-enumeration positions, column ids = Ad row positions).
void build_stencil_operator(System& S) {
    hipStream_t st = S.stream;
    const int64_t npts = S.mfh.npts, nf = S.n_full, n = S.G.n;
    S.keep.alloc(std::max<int64_t>(n, 1));
    hipLaunchKernelGGL(k_keep_list, dim3(grid_for(nf)), dim3(BLOCK), 0, st, nf, S.have_colmap ? S.colmap.p : nullptr,
                       S.keep.p);
    KERNEL_CHECK();
    DBuf<int32_t> inv;
    locality_order(S.G, npts, npts, S.Ad.perm, inv, st);
    build_sell(S.Ad, S.G, npts, S.keep.p, st);
    transpose_rows(S.G, npts, S.GdT, st);
    // ATd row = node-enumeration position (MfDesc): GdT row of its column, -1 for alignment
    // padding and removed columns
    S.mfd.alloc(1);
    S.mfd.upload(&S.mfh, 1, st);
    const int64_t ne = S.mfh.nodes;
    S.ATd.perm.alloc(std::max<int64_t>(ne, 1));
    hipLaunchKernelGGL(k_enum_perm, dim3(grid_for(ne)), dim3(BLOCK), 0, st, S.mfd.p, ne,
                       S.have_colmap ? S.colmap.p : nullptr, S.ATd.perm.p);
    KERNEL_CHECK();
    build_csr32(S.ATd, S.GdT, ne, inv.p, st);
    S.csf.alloc(std::max<int64_t>(nf, 1));
    S.zv.alloc(std::max<int64_t>(nf, 1));
    S.zv.zero(st);
    HIP_CHECK(hipStreamSynchronize(st));
}

}  // namespace

void finish_formation(System& S) {
    S.dmf = DmfDesc{};
    hipStream_t st = S.stream;
    Csr& G = S.G;
    const int64_t m = G.m, n = G.n;
    if (S.g_full) transpose_rows(G, m, S.GT, st);   // lazy structured formation: GT with the full G
    S.sell_built = false;
    S.A = Sell();
    S.AT = Sell();
    if (S.mf)
        build_stencil_operator(S);
    else
        ensure_sell(S);

    // default scaling state: weights 1, all rows kept, no preconditioner
    S.roww.alloc(m);
    hipLaunchKernelGGL(k_fill, dim3(grid_for(m)), dim3(BLOCK), 0, st, m, 1.0, S.roww.p);
    KERNEL_CHECK();
    S.rowkeep.alloc(m);
    HIP_CHECK(hipMemsetAsync(S.rowkeep.p, 1, m, st));
    S.rs.alloc(m);
    S.cs.alloc(std::max<int64_t>(n, 1));
    S.rs_dirty = true;
    S.cs_mode = -1;
    S.iter_ready = false;
    S.nblk = 0;   // column blocks refer to the previous column numbering
    S.blk_user = false;
    S.blk_valid = false;
    HIP_CHECK(hipStreamSynchronize(st));
}

void full_transpose(System& S) {
    transpose_rows(S.G, S.G.m, S.GT, S.stream);
    HIP_CHECK(hipStreamSynchronize(S.stream));
}

// Scaling is applied in three phases so a distributed group can exchange column norms between
// them: (1) row scale + (raw) column norms, (2) [dist: reverse halo, finish, forward halo],
// (3) fill the SELL values.
void scaling_rows_colnorm(System& S, int precond, bool raw) {
    hipStream_t st = S.stream;
    const int64_t m = S.G.m, n = S.G.n;
    hipLaunchKernelGGL(k_rowscale, dim3(grid_for(m)), dim3(BLOCK), 0, st, m, S.roww.p, S.rowkeep.p, S.rs.p);
    KERNEL_CHECK();
    S.dense_valid = false;   // the dense, band and block factors depend on the row scaling
    S.band.valid = false;
    S.blk_valid = false;
    if (precond == 1 && S.mf)
        mf_column_scale(S, raw);
    else if (precond == 1)
        hipLaunchKernelGGL(k_colnorm, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, S.GT.rp.p, S.GT.ci.p, S.GT.val.p,
                           S.rs.p, S.cs.p, raw ? 1 : 0);
    else
        hipLaunchKernelGGL(k_fill, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, 1.0, S.cs.p);
    KERNEL_CHECK();
}

void scaling_finish_cs(System& S) {
    hipLaunchKernelGGL(k_cs_finish, dim3(grid_for(S.n_own)), dim3(BLOCK), 0, S.stream, S.n_own, S.cs.p);
    KERNEL_CHECK();
}

void scaling_fill_values(System& S, int precond, bool set_csf) {
    hipStream_t st = S.stream;
    const int64_t m = S.G.m, n = S.G.n;
    if (S.sell_built) {
        hipLaunchKernelGGL(k_sell_vals, dim3(grid_for(m)), dim3(BLOCK), 0, st, m, S.G.rp.p, S.G.ci.p, S.G.val.p,
                           S.rs.p, S.cs.p, 0, S.A.perm.p, S.A.sp.p, S.A.val.p);
        KERNEL_CHECK();
        hipLaunchKernelGGL(k_sell_vals, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, S.GT.rp.p, S.GT.ci.p, S.GT.val.p,
                           S.rs.p, S.cs.p, 1, nullptr, S.AT.sp.p, S.AT.val.p);
        KERNEL_CHECK();
    }
    if (S.mf) {   // data rows carry the row scale only; the stencil kernels apply cs themselves
        const int64_t npts = S.mfh.npts;
        hipLaunchKernelGGL(k_sell_vals, dim3(grid_for(npts)), dim3(BLOCK), 0, st, npts, S.G.rp.p, S.G.ci.p,
                           S.G.val.p, S.rs.p, nullptr, 0, S.Ad.perm.p, S.Ad.sp.p, S.Ad.val.p);
        KERNEL_CHECK();
        hipLaunchKernelGGL(k_c32_vals, dim3(grid_for(S.ATd.rows)), dim3(BLOCK), 0, st, S.ATd.rows, S.ATd.perm.p,
                           S.GdT.rp.p, S.GdT.ci.p, S.GdT.val.p, S.rs.p, S.ATd.rp.p, S.ATd.val.p);
        KERNEL_CHECK();
        if (set_csf) {   // distributed ranks assemble csf themselves (column norms span ranks)
            S.csf.zero(st);
            hipLaunchKernelGGL(k_scatter_cs, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, S.keep.p, S.cs.p, S.csf.p);
            KERNEL_CHECK();
        }
        // parts whose rows share one row scale skip the per-row scale loads in the iteration
        const int np = S.mfh.n_parts;
        const int nc = np * MINMAX_CHUNKS;
        DBuf<double> mm(2 * nc);
        hipLaunchKernelGGL(k_part_minmax, dim3(nc), dim3(BLOCK), 0, st, S.mfd.p, S.rs.p, mm.p);
        KERNEL_CHECK();
        std::vector<double> h(2 * nc);
        mm.download(h.data(), 2 * nc, st);
        HIP_CHECK(hipStreamSynchronize(st));
        for (int p = 0; p < np; ++p) {
            double lo = INFINITY, hi = -INFINITY;
            for (int c = 0; c < MINMAX_CHUNKS; ++c) {
                lo = std::min(lo, h[2 * (p * MINMAX_CHUNKS + c)]);
                hi = std::max(hi, h[2 * (p * MINMAX_CHUNKS + c) + 1]);
            }
            S.mfh.p[p].wconst = lo == hi ? 1 : 0;
            S.mfh.p[p].w = lo;
        }
        S.mfd.upload(&S.mfh, 1, st);
    }
    S.rs_dirty = false;
    S.cs_mode = precond;
    S.iter_ready = false;
}

// row mask from the host (any non-zero byte keeps the row): uploaded as given, 0/1 on the device
void upload_row_mask(System& S, const uint8_t* keep) {
    if (keep) {
        S.rowkeep.upload(keep, S.G.m, S.stream);
        hipLaunchKernelGGL(k_mask01, dim3(grid_for(S.G.m)), dim3(BLOCK), 0, S.stream, S.G.m, S.rowkeep.p);
        KERNEL_CHECK();
    } else {
        HIP_CHECK(hipMemsetAsync(S.rowkeep.p, 1, S.G.m, S.stream));
    }
    HIP_CHECK(hipStreamSynchronize(S.stream));
}

bool scaling_stale(const System& S, int precond) { return S.rs_dirty || S.cs_mode != precond; }

void refresh_scaling(System& S, int precond) {
    if (!scaling_stale(S, precond)) return;
    if (S.dist) throw std::logic_error("refresh_scaling: distributed systems refresh through their group");
    scaling_rows_colnorm(S, precond, false);
    scaling_fill_values(S, precond);
}

void csr_spmv(System& S, int trans, const double* dx, double* dy) {
    ensure_full_csr(S);
    const Csr& C = trans ? S.GT : S.G;
    hipLaunchKernelGGL(k_csr_spmv, dim3(grid_for(C.m)), dim3(BLOCK), 0, S.stream, C.m, C.rp.p, C.ci.p, C.val.p, dx, dy);
    KERNEL_CHECK();
}

void csr_spmv_rows(System& S, int64_t first, int64_t count, const double* dx, double* dy) {
    if (!count) return;
    if (first + count > stored_rows(S)) ensure_full_csr(S);
    hipLaunchKernelGGL(k_csr_spmv, dim3(grid_for(count)), dim3(BLOCK), 0, S.stream, count, S.G.rp.p + first, S.G.ci.p,
                       S.G.val.p, dx, dy);
    KERNEL_CHECK();
}

void csr_rows_sumsq(System& S, const double* dx, int64_t first, int64_t count, double* h_w, double* h_u) {
    const int nb = grid_for(std::max<int64_t>(count, 1));
    DBuf<double> pw(nb), pu(nb);
    const int64_t ns = stored_rows(S);
    if (first + count <= ns) {
        hipLaunchKernelGGL(k_rows_sumsq, dim3(nb), dim3(BLOCK), 0, S.stream, first, count, S.G.rp.p, S.G.ci.p, S.G.val.p,
                           dx, S.roww.p, pw.p, pu.p);
    } else if (first >= ns) {   // stencil rows of a lazily formed system: from the part descriptors
        DBuf<double> xf(std::max<int64_t>(S.n_full, 1));
        xf.zero(S.stream);
        hipLaunchKernelGGL(k_scatter_cs, dim3(grid_for(S.G.n)), dim3(BLOCK), 0, S.stream, S.G.n, S.keep.p, dx, xf.p);
        hipLaunchKernelGGL(k_rows_sumsq_mf, dim3(nb), dim3(BLOCK), 0, S.stream, S.mfd.p, first, count, xf.p, S.roww.p,
                           pw.p, pu.p);
    } else {   // a range across the data / stencil boundary: the two pieces
        double w1, u1, w2, u2;
        csr_rows_sumsq(S, dx, first, ns - first, &w1, &u1);
        csr_rows_sumsq(S, dx, ns, first + count - ns, &w2, &u2);
        *h_w = w1 + w2;
        *h_u = u1 + u2;
        return;
    }
    KERNEL_CHECK();
    std::vector<double> hw(nb), hu(nb);
    pw.download(hw.data(), nb, S.stream);
    pu.download(hu.data(), nb, S.stream);
    HIP_CHECK(hipStreamSynchronize(S.stream));
    double a = 0.0, b = 0.0;   // fixed order: deterministic
    for (int i = 0; i < nb; ++i) {
        a += hw[i];
        b += hu[i];
    }
    *h_w = a;
    *h_u = b;
}

void referenced_cols(System& S, uint8_t* h_flags) {
    ensure_full_csr(S);
    DBuf<uint8_t> f(std::max<int64_t>(S.G.n, 1));
    f.zero(S.stream);
    hipLaunchKernelGGL(k_flag_cols, dim3(grid_for(S.G.nnz)), dim3(BLOCK), 0, S.stream, S.G.nnz, S.G.ci.p, f.p);
    KERNEL_CHECK();
    f.download(h_flags, S.G.n, S.stream);
    HIP_CHECK(hipStreamSynchronize(S.stream));
}

void relabel_columns(System& S, const int32_t* h_map, int64_t n_local) {
    ensure_full_csr(S);
    S.gen_ctx.clear();   // G no longer regenerates from the formation (release_full_csr refuses)
    S.dmf.ok = 0;   // the matrix-free data rows address the formation's column space
    DBuf<int32_t> map(std::max<int64_t>(S.G.n, 1));
    map.upload(h_map, S.G.n, S.stream);
    DBuf<unsigned long long> bad(1);
    bad.zero(S.stream);
    hipLaunchKernelGGL(k_relabel_rows, dim3(grid_for(S.G.m)), dim3(BLOCK), 0, S.stream, S.G.m, S.G.rp.p, S.G.ci.p,
                       S.G.val.p, map.p, bad.p);
    KERNEL_CHECK();
    unsigned long long h = 0;
    HIP_CHECK(hipMemcpyAsync(&h, bad.p, sizeof(h), hipMemcpyDeviceToHost, S.stream));
    HIP_CHECK(hipStreamSynchronize(S.stream));
    if (h) throw std::invalid_argument("lsq_dist_set_layout: a referenced column has no local index");
    S.G.n = n_local;
    S.GT = Csr{};
    S.mf = false;   // distributed ranks stream the assembled local operator
    S.Ad = Sell{};
    S.ATd = Csr32{};
    S.GdT = Csr{};
    finish_formation(S);
}

System::~System() {
    mg_free(mg);
    delete mx;
    if (comm) (void)ncclCommDestroy(comm);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (side) (void)hipStreamDestroy(side);
    if (ev_aux) (void)hipEventDestroy(ev_aux);
    if (aux) (void)hipStreamDestroy(aux);
    if (aux_side) (void)hipStreamDestroy(aux_side);
    if (stream && own_stream) (void)hipStreamDestroy(stream);
}

}  // namespace lsq
