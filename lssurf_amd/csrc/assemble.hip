// assemble.hip — structured device formation of the smooth_fit operator (no host triplets).
//
// One thread generates one row of [G_data; Gc] exactly as the host lin_op would:
//   data row p   : Σ over interpolation parts of the 2^ndim bi/trilinear weights of point p
//                  (lin_op.interp_mtx, lin_op.py:163-247: f = (p-b0)/δ, cell = floor(f),
//                  w = ((1·a0)·a1)·a2 with a_d = f_d - cell_d or 1-(f_d - cell_d), corners in
//                  np.mgrid order)
//   stencil row  : centre = lo + unravel(k, hi-lo) in 'ij' meshgrid order, entries
//                  col0 + ravel(centre + off_t) with value val_t (lin_op.diff_op, lin_op.py:80-132)
// then drops v == 0, removes Ip_c columns, sorts by (column, generation order), sums duplicates
// and drops zero sums — the same rules as the COO path — and writes canonical CSR.  Two passes
// (count, fill) around an exclusive scan.  Compiled with -ffp-contract=off: the weights are
// bit-identical to numpy's.
#include <algorithm>
#include <vector>

#include "../../include/lsqsurf.h"
#include "system.hpp"

namespace lsq {
namespace {

constexpr int MAX_GRIDS = 4, MAX_INTERP = 4, MAX_STENCIL = 32, MAXE = 32;

struct GenCtx {
    int32_t n_grids, n_interp, n_stencil, pad;
    int64_t npts, m, n_full;
    lsq_grid_desc grids[MAX_GRIDS];
    int64_t stride[MAX_GRIDS][3];
    int32_t interp_grid[MAX_INTERP];
    lsq_stencil_desc st[MAX_STENCIL];
};

__global__ __launch_bounds__(BLOCK) void k_gen_rows(int pass, const GenCtx* __restrict__ ctx,
                                                    const double* __restrict__ py, const double* __restrict__ px,
                                                    const double* __restrict__ pt, const int32_t* __restrict__ colmap,
                                                    int64_t* __restrict__ cnt, const int64_t* __restrict__ rp,
                                                    int32_t* __restrict__ ci, double* __restrict__ val,
                                                    unsigned long long* __restrict__ err) {
    const int64_t m = ctx->m;
    for (int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x; r < m; r += (int64_t)gridDim.x * BLOCK) {
        int64_t cols[MAXE];
        double vals[MAXE];
        int ne = 0;
        if (r < ctx->npts) {
            const double p[3] = {py[r], px[r], pt ? pt[r] : 0.0};
            for (int k = 0; k < ctx->n_interp; ++k) {
                const int gi = ctx->interp_grid[k];
                const lsq_grid_desc& g = ctx->grids[gi];
                const int nd = g.ndim;
                double fr[3];
                int64_t base = 0;
                for (int d = 0; d < nd; ++d) {
                    const double f = (p[d] - g.b0[d]) / g.delta[d];
                    const double cf = floor(f);
                    fr[d] = f - cf;
                    base = base * g.shape[d] + (int64_t)cf;
                }
                base += g.col0;
                const int ncorner = 1 << nd;
                for (int q = 0; q < ncorner && ne < MAXE; ++q) {
                    int64_t col = base;
                    double w = 1.0;
                    for (int d = 0; d < nd; ++d) {
                        const int bit = (q >> (nd - 1 - d)) & 1;
                        col += bit * ctx->stride[gi][d];
                        w *= bit ? fr[d] : (1. - fr[d]);
                    }
                    cols[ne] = col;
                    vals[ne] = w;
                    ++ne;
                }
            }
        } else {
            int s = 0;
            while (s + 1 < ctx->n_stencil && r >= ctx->st[s + 1].row0) ++s;
            const lsq_stencil_desc& S = ctx->st[s];
            const lsq_grid_desc& g = ctx->grids[S.grid];
            const int nd = g.ndim;
            int64_t rem = r - S.row0;
            int64_t sub[3] = {0, 0, 0};
            for (int d = nd - 1; d >= 0; --d) {
                const int64_t ext = S.hi[d] - S.lo[d];
                sub[d] = S.lo[d] + rem % ext;
                rem /= ext;
            }
            for (int t = 0; t < S.ntpl && ne < MAXE; ++t) {
                int64_t col = g.col0;
                for (int d = 0; d < nd; ++d) col += (sub[d] + S.off[t][d]) * ctx->stride[S.grid][d];
                cols[ne] = col;
                vals[ne] = S.val[t];
                ++ne;
            }
        }
        // toCSR / Ip_c rules: drop zeros, drop removed columns (generation order preserved)
        int nk = 0;
        for (int e = 0; e < ne; ++e) {
            if (vals[e] == 0.0) continue;
            int64_t c = cols[e];
            if (c < 0 || c >= ctx->n_full) {
                atomicAdd(err, 1ull);
                continue;
            }
            if (colmap) {
                c = colmap[c];
                if (c < 0) continue;
            }
            cols[nk] = c;
            vals[nk] = vals[e];
            ++nk;
        }
        // stable insertion sort by column
        for (int i = 1; i < nk; ++i) {
            const int64_t kc = cols[i];
            const double kv = vals[i];
            int j = i - 1;
            while (j >= 0 && cols[j] > kc) {
                cols[j + 1] = cols[j];
                vals[j + 1] = vals[j];
                --j;
            }
            cols[j + 1] = kc;
            vals[j + 1] = kv;
        }
        int out = 0;
        const int64_t o = pass ? rp[r] : 0;
        for (int i = 0; i < nk;) {
            const int64_t c = cols[i];
            double sum = vals[i];
            int k = i + 1;
            while (k < nk && cols[k] == c) sum += vals[k++];
            if (sum != 0.0) {
                if (pass) {
                    ci[o + out] = (int32_t)c;
                    val[o + out] = sum;
                }
                ++out;
            }
            i = k;
        }
        if (!pass) cnt[r] = out;
    }
}

}  // namespace

void form_from_stencils(System& S, int64_t m, int64_t n_full, int32_t n_grids, const lsq_grid_desc* grids,
                        int32_t n_interp, const int32_t* interp_grid, int64_t npts, const double* py,
                        const double* px, const double* pt, int32_t n_stencil, const lsq_stencil_desc* st) {
    if (n_grids < 1 || n_grids > MAX_GRIDS || n_interp < 0 || n_interp > MAX_INTERP || n_stencil < 0 ||
        n_stencil > MAX_STENCIL)
        throw std::invalid_argument("lsq_set_matrix_stencil: too many grids / parts");
    GenCtx h{};
    h.n_grids = n_grids;
    h.n_interp = n_interp;
    h.n_stencil = n_stencil;
    h.npts = npts;
    h.m = m;
    h.n_full = n_full;
    bool need_t = false;
    for (int g = 0; g < n_grids; ++g) {
        h.grids[g] = grids[g];
        if (grids[g].ndim < 1 || grids[g].ndim > 3) throw std::invalid_argument("grid ndim must be 1..3");
        int64_t s = 1;
        for (int d = grids[g].ndim - 1; d >= 0; --d) {
            h.stride[g][d] = s;
            s *= grids[g].shape[d];
        }
    }
    int ncorners = 0;
    for (int k = 0; k < n_interp; ++k) {
        if (interp_grid[k] < 0 || interp_grid[k] >= n_grids) throw std::invalid_argument("bad interp grid");
        h.interp_grid[k] = interp_grid[k];
        need_t |= grids[interp_grid[k]].ndim == 3;
        ncorners += 1 << grids[interp_grid[k]].ndim;
    }
    if (ncorners > MAXE) throw std::invalid_argument("too many interpolation corners per row");
    int64_t expect = npts;
    for (int s = 0; s < n_stencil; ++s) {
        h.st[s] = st[s];
        if (st[s].grid < 0 || st[s].grid >= n_grids || st[s].ntpl < 1 || st[s].ntpl > 8)
            throw std::invalid_argument("bad stencil descriptor");
        if (st[s].row0 != expect) throw std::invalid_argument("stencil parts must tile rows [npts, m) in order");
        int64_t ext = 1;
        for (int d = 0; d < grids[st[s].grid].ndim; ++d) ext *= std::max<int64_t>(st[s].hi[d] - st[s].lo[d], 0);
        if (ext != st[s].n_eq) throw std::invalid_argument("stencil n_eq does not match its centre box");
        expect += st[s].n_eq;
    }
    if (expect != m) throw std::invalid_argument("rows of the parts do not add up to m");
    if (npts > 0 && (!py || !px || (need_t && !pt))) throw std::invalid_argument("missing point coordinates");

    hipStream_t strm = S.stream;
    const int64_t n = S.have_colmap ? S.n_keep : n_full;
    DBuf<GenCtx> dctx(1);
    HIP_CHECK(hipMemcpyAsync(dctx.p, &h, sizeof(GenCtx), hipMemcpyHostToDevice, strm));
    DBuf<double> dy(std::max<int64_t>(npts, 1)), dx(std::max<int64_t>(npts, 1)), dt;
    dy.upload(py, npts, strm);
    dx.upload(px, npts, strm);
    if (need_t) {
        dt.alloc(std::max<int64_t>(npts, 1));
        dt.upload(pt, npts, strm);
    }
    DBuf<unsigned long long> err(1);
    err.zero(strm);
    Csr& G = S.G;
    G.m = m;
    G.n = n;
    G.rp.alloc(m + 1);
    G.rp.zero(strm);
    const int32_t* cmap = S.have_colmap ? S.colmap.p : nullptr;
    const int grid = grid_for(m);
    hipLaunchKernelGGL(k_gen_rows, dim3(grid), dim3(BLOCK), 0, strm, 0, dctx.p, dy.p, dx.p, dt.p, cmap, G.rp.p,
                       nullptr, nullptr, nullptr, err.p);
    KERNEL_CHECK();
    G.nnz = exclusive_scan_i64(G.rp.p, m + 1, strm);
    G.ci.alloc(std::max<int64_t>(G.nnz, 1));
    G.val.alloc(std::max<int64_t>(G.nnz, 1));
    hipLaunchKernelGGL(k_gen_rows, dim3(grid), dim3(BLOCK), 0, strm, 1, dctx.p, dy.p, dx.p, dt.p, cmap, nullptr,
                       G.rp.p, G.ci.p, G.val.p, err.p);
    KERNEL_CHECK();
    unsigned long long herr = 0;
    HIP_CHECK(hipMemcpyAsync(&herr, err.p, sizeof(herr), hipMemcpyDeviceToHost, strm));
    HIP_CHECK(hipStreamSynchronize(strm));
    if (herr) throw std::invalid_argument("lsq_set_matrix_stencil: " + std::to_string(herr) +
                                          " nonzero entries fall outside [0, n_full)");
    S.n_sorted_rows = npts;   // data rows: point order is random in space
    finish_formation(S);
}

}  // namespace lsq
