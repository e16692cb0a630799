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
#include <cmath>
#include <cstdlib>
#include <vector>

#include "../../include/lsqsurf.h"
#include "system.hpp"

namespace lsq {
namespace {

constexpr int MAX_GRIDS = 4, MAX_INTERP = 4, MAX_STENCIL = 32, MAXE = 32;

// one stencil part as the formation sees it: lsq_stencil_desc, or its field-valued override
// (lsq_set_stencil_fields: ≤ MF_MAXT entries, value val[t] · F[fsel[t]·n_eq + k] for centre k)
struct GenSt {
    int32_t grid, ntpl;
    int32_t off[MF_MAXT][3];
    double val[MF_MAXT];
    int32_t fsel[MF_MAXT];
    int64_t row0, n_eq;
    int64_t lo[3], hi[3];
    const double* F;   // null: constant values
};

struct GenCtx {
    int32_t n_grids, n_interp, n_stencil, pad;
    int64_t npts, m, n_full;
    lsq_grid_desc grids[MAX_GRIDS];
    int64_t stride[MAX_GRIDS][3];
    int32_t interp_grid[MAX_INTERP];
    GenSt st[MAX_STENCIL];
};

__global__ __launch_bounds__(BLOCK) void k_gen_rows(int pass, const GenCtx* __restrict__ ctx,
                                                    const double* __restrict__ py, const double* __restrict__ px,
                                                    const double* __restrict__ pt, const int32_t* __restrict__ colmap,
                                                    int64_t* __restrict__ cnt, const int64_t* __restrict__ rp,
                                                    int32_t* __restrict__ ci, double* __restrict__ val,
                                                    unsigned long long* __restrict__ err, int64_t m,
                                                    const uint8_t* __restrict__ keep = nullptr,
                                                    unsigned long long* __restrict__ ksum = nullptr) {
    // ksum (count pass, lsq_shape of a lazily formed system): instead of cnt, the kept rows and
    // their entries are summed into ksum[0], ksum[1] (keep[r] != 0: row r kept)
    double kr = 0.0, kz = 0.0;
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
            const GenSt& S = ctx->st[s];
            const lsq_grid_desc& g = ctx->grids[S.grid];
            const int nd = g.ndim;
            const int64_t k = r - S.row0;
            int64_t rem = k;
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
                vals[ne] = S.F ? S.val[t] * S.F[S.fsel[t] * S.n_eq + k] : S.val[t];
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
        if (ksum) {
            if (keep[r]) {
                kr += 1.0;
                kz += (double)out;
            }
        } else if (!pass) {
            cnt[r] = out;
        }
    }
    if (ksum) {   // exact: every partial count is far below 2^53
        kr = wave_sum(kr);
        kz = wave_sum(kz);
        if ((threadIdx.x & 63) == 0 && kr > 0.0) {
            atomicAdd(ksum, (unsigned long long)kr);
            atomicAdd(ksum + 1, (unsigned long long)kz);
        }
    }
}


// The structured stencil operator (system.hpp MfDesc) when every part is a clean stencil:
// every template entry of every centre in the box stays inside its grid, grids do not overlap,
// and every index fits 31 bits.
bool describe_stencil_operator(MfDesc& d, int64_t m, int64_t n_full, int32_t n_grids, const lsq_grid_desc* grids,
                               int64_t npts, int32_t n_stencil, const GenSt* st) {
    d = MfDesc{};
    d.npts = npts;
    d.m = m;
    d.n_full = n_full;
    if (n_grids > MF_MAX_GRIDS || m >= (int64_t(1) << 31) || n_full >= (int64_t(1) << 31)) return false;
    for (int g = 0; g < n_grids; ++g) {
        MfGrid& G = d.g[g];
        G.ndim = 3;   // every grid is padded to 3 dims with trailing extent-1 dims (same ravel)
        G.col0 = (int32_t)grids[g].col0;
        int64_t s = 1;
        for (int k = 2; k >= 0; --k) {
            G.shape[k] = k < grids[g].ndim ? (int32_t)grids[g].shape[k] : 1;
            G.fd[k] = make_fastdiv((uint32_t)std::max<int32_t>(G.shape[k], 1));
            s *= G.shape[k];
        }
        G.nodes = (int32_t)s;
        if (grids[g].col0 < 0 || grids[g].col0 + s > n_full) return false;
        for (int h = 0; h < g; ++h)
            if (G.col0 < d.g[h].col0 + d.g[h].nodes && d.g[h].col0 < G.col0 + s) return false;
    }
    d.n_grids = n_grids;
    for (int i = 0; i < n_stencil; ++i) {
        const GenSt& S = st[i];
        if (S.n_eq == 0) continue;
        if (d.n_parts == MF_MAX_PARTS) return false;
        MfGrid& G = d.g[S.grid];
        if (G.nparts == MF_MAX_GRID_PARTS) return false;
        MfPart& P = d.p[d.n_parts];
        P.grid = S.grid;
        P.ntpl = S.ntpl;
        P.row0 = (int32_t)S.row0;
        P.n_eq = (int32_t)S.n_eq;
        const int nd = grids[S.grid].ndim;
        int64_t bs = 1, gs = 1;
        int64_t stride[3];
        for (int k = 2; k >= 0; --k) {
            P.lo[k] = k < nd ? (int32_t)S.lo[k] : 0;
            P.hi[k] = k < nd ? (int32_t)S.hi[k] : 1;
            P.bstride[k] = (int32_t)bs;
            stride[k] = gs;
            bs *= P.hi[k] - P.lo[k];
            gs *= G.shape[k];
        }
        for (int k = 0; k < 3; ++k) {
            P.ilo[k] = P.lo[k];
            P.ihi[k] = P.hi[k];
        }
        for (int t = 0; t < S.ntpl; ++t) {
            P.doff[t] = P.boff[t] = 0;
            for (int k = 0; k < 3; ++k) {
                const int64_t o = k < nd ? S.off[t][k] : 0;
                if (P.lo[k] + o < 0 || P.hi[k] - 1 + o >= G.shape[k] || o < -MF_R || o > MF_R) return false;
                P.off[t][k] = (int32_t)o;
                P.doff[t] += (int32_t)(o * stride[k]);
                P.boff[t] += (int32_t)(o * P.bstride[k]);
                P.ilo[k] = std::max<int32_t>(P.ilo[k], P.lo[k] + (int32_t)o);
                P.ihi[k] = std::min<int32_t>(P.ihi[k], P.hi[k] + (int32_t)o);
            }
            P.val[t] = S.val[t];
            P.fsel[t] = S.F ? S.fsel[t] : 0;
        }
        P.var = S.F ? 1 : 0;
        P.F = S.F;
        P.nfield = 0;
        for (int t = 0; t < S.ntpl; ++t) P.nfield = std::max(P.nfield, P.fsel[t] + 1);
        // Aᵀu validity of template t for a column c: lo <= c - off_t < hi in every dim, i.e.
        // off_t <= c - lo and off_t >= c - hi + 1.  With |off| <= MF_R both sides depend only on
        // a = clamp(c - lo + MF_R + 1, 0, 2 MF_R + 1) and b = clamp(c - hi + MF_R + 1, ...):
        // mlo[k][a] / mhi[k][b] hold the templates valid on that side (bit t).
        for (int k = 0; k < 3; ++k) {
            P.mlo[k][0] = P.mlo[k][1] = P.mhi[k][0] = P.mhi[k][1] = P.mlo8[k] = P.mhi8[k] = 0;
            for (int a = 0; a <= 2 * MF_R + 1; ++a) {
                uint64_t lo_bits = 0, hi_bits = 0;
                for (int t = 0; t < S.ntpl; ++t) {
                    if (P.off[t][k] <= a - MF_R - 1) lo_bits |= uint64_t(1) << t;
                    if (P.off[t][k] >= a - MF_R) hi_bits |= uint64_t(1) << t;
                }
                P.mlo[k][a >> 2] |= lo_bits << (16 * (a & 3));
                P.mhi[k][a >> 2] |= hi_bits << (16 * (a & 3));
                P.mlo8[k] |= (lo_bits & 0xFF) << (8 * a);
                P.mhi8[k] |= (hi_bits & 0xFF) << (8 * a);
            }
        }
        G.part[G.nparts++] = d.n_parts++;
    }
    // A·v LDS bands per grid: one per distinct template y offset, spanning its in-row offsets
    for (int g = 0; g < n_grids; ++g) {
        MfGrid& G = d.g[g];
        int emin[2 * MF_R + 1], emax[2 * MF_R + 1], band_of[2 * MF_R + 1];
        bool used[2 * MF_R + 1] = {};
        for (int q = 0; q < G.nparts; ++q) {
            const MfPart& P = d.p[G.part[q]];
            for (int t = 0; t < P.ntpl; ++t) {
                const int oy = P.off[t][0] + MF_R, e = P.off[t][1] * G.shape[2] + P.off[t][2];
                if (!used[oy]) emin[oy] = emax[oy] = e;
                used[oy] = true;
                emin[oy] = std::min(emin[oy], e);
                emax[oy] = std::max(emax[oy], e);
            }
        }
        G.nband = 0;
        G.lds = 0;
        for (int oy = 0; oy <= 2 * MF_R; ++oy) {
            if (!used[oy]) continue;
            const int b = G.nband++;
            band_of[oy] = b;
            G.band_oy[b] = oy - MF_R;
            G.band_emin[b] = emin[oy];
            G.band_len[b] = MF_ALIGN + emax[oy] - emin[oy];
            G.band_start[b] = G.lds;
            G.lds += G.band_len[b];
        }
        if (G.lds > MF_LDS_MAX) G.lds = 0;   // too wide: the A·v kernel gathers from HBM
        for (int q = 0; q < G.nparts; ++q) {
            MfPart& P = d.p[G.part[q]];
            for (int t = 0; t < P.ntpl; ++t) {
                const int b = band_of[P.off[t][0] + MF_R];
                P.loff[t] = G.band_start[b] + P.off[t][1] * G.shape[2] + P.off[t][2] - G.band_emin[b];
            }
        }
    }
    // node enumeration: the grids with parts, each starting on a MF_ALIGN boundary, so a block
    // iteration (A·v) or a wave's 256 columns (Aᵀu) never spans two grids; they must cover every
    // column (the Aᵀu kernel walks this enumeration)
    int64_t node0 = 0, covered = 0;
    for (int g = 0; g < n_grids; ++g) {
        d.g[g].node0 = (int32_t)node0;
        if (d.g[g].nparts) {
            node0 += (d.g[g].nodes + MF_ALIGN - 1) / MF_ALIGN * MF_ALIGN;
            covered += d.g[g].nodes;
        }
    }
    d.nodes = node0;
    return d.n_parts > 0 && covered == n_full && node0 < (int64_t(1) << 31);
}

GenSt gen_of(const lsq_stencil_desc& d) {
    GenSt G{};
    G.grid = d.grid;
    G.ntpl = d.ntpl;
    G.row0 = d.row0;
    G.n_eq = d.n_eq;
    for (int k = 0; k < 3; ++k) {
        G.lo[k] = d.lo[k];
        G.hi[k] = d.hi[k];
    }
    G.F = nullptr;
    for (int t = 0; t < std::min(d.ntpl, 8); ++t) {
        for (int k = 0; k < 3; ++k) G.off[t][k] = d.off[t][k];
        G.val[t] = d.val[t];
    }
    return G;
}

}  // namespace

// The global structure behind a rank's window (host only, for the distributed multigrid's coarse
// levels): grids and stencil parts as describe_stencil_operator sees them; parts with ntpl = 0 are
// field-valued (their coarse rows come from the ranks' partial Galerkin rows).
void describe_global(System& S, int64_t n_full, int32_t n_grids, const lsq_grid_desc* grids, int32_t n_stencil,
                     const lsq_stencil_desc* st) {
    if (n_grids < 1 || n_grids > MAX_GRIDS || n_stencil < 0 || n_stencil > MAX_STENCIL)
        throw std::invalid_argument("lsq_dist_set_global: too many grids / parts");
    std::vector<GenSt> gs(n_stencil);
    int64_t m = 0, npts = 0;
    for (int s = 0; s < n_stencil; ++s) {
        gs[s] = gen_of(st[s]);
        if (st[s].ntpl < 0 || st[s].ntpl > 8) throw std::invalid_argument("lsq_dist_set_global: bad stencil");
        m = std::max<int64_t>(m, st[s].row0 + st[s].n_eq);
    }
    MfDesc d{};
    if (!describe_stencil_operator(d, m, n_full, n_grids, grids, npts, n_stencil, gs.data()))
        throw std::invalid_argument("lsq_dist_set_global: the global parts are not a structured stencil operator");
    int q = 0;
    for (int s = 0; s < n_stencil; ++s) {   // describe_stencil_operator keeps the non-empty parts in order
        if (st[s].n_eq == 0) continue;
        d.p[q].var = st[s].ntpl == 0 ? 1 : 0;
        ++q;
    }
    S.dg_mfh = d;
}

namespace {

// G's row pointers for all m rows (count pass: validates every row and gives the formed nnz), then
// the entries of the first `rows` rows (fill pass).  S.G.m = m either way; rows < m keeps npts + 1
// row pointers (the lazy structured formation: rows = the data rows).
void gen_rows_csr(System& S, const double* dy, const double* dx, const double* dt, int64_t rows) {
    hipStream_t strm = S.stream;
    const GenCtx& h = *reinterpret_cast<const GenCtx*>(S.gen_ctx.data());
    const int64_t m = h.m;
    DBuf<GenCtx> dctx(1);
    HIP_CHECK(hipMemcpyAsync(dctx.p, &h, sizeof(GenCtx), hipMemcpyHostToDevice, strm));
    DBuf<unsigned long long> err(1);
    err.zero(strm);
    const int32_t* cmap = S.have_colmap ? S.colmap.p : nullptr;
    DBuf<int64_t> rp(m + 1);
    rp.zero(strm);
    hipLaunchKernelGGL(k_gen_rows, dim3(grid_for(m)), dim3(BLOCK), 0, strm, 0, dctx.p, dy, dx, dt, cmap, rp.p, nullptr,
                       nullptr, nullptr, err.p, m);
    KERNEL_CHECK();
    S.nnz_full = exclusive_scan_i64(rp.p, m + 1, strm);
    Csr& G = S.G;
    G.m = m;
    G.n = S.have_colmap ? S.n_keep : h.n_full;
    if (rows < m) {
        G.rp.alloc(rows + 1);
        HIP_CHECK(hipMemcpyAsync(G.rp.p, rp.p, sizeof(int64_t) * (rows + 1), hipMemcpyDeviceToDevice, strm));
        HIP_CHECK(hipMemcpyAsync(&G.nnz, rp.p + rows, sizeof(int64_t), hipMemcpyDeviceToHost, strm));
        HIP_CHECK(hipStreamSynchronize(strm));   // rp is released below
    } else {
        G.rp = std::move(rp);
        G.nnz = S.nnz_full;
    }
    G.ci.alloc(std::max<int64_t>(G.nnz, 1));
    G.val.alloc(std::max<int64_t>(G.nnz, 1));
    if (rows > 0)
        hipLaunchKernelGGL(k_gen_rows, dim3(grid_for(rows)), dim3(BLOCK), 0, strm, 1, dctx.p, dy, dx, dt, cmap, nullptr,
                           G.rp.p, G.ci.p, G.val.p, err.p, rows);
    KERNEL_CHECK();
    unsigned long long herr = 0;
    HIP_CHECK(hipMemcpyAsync(&herr, err.p, sizeof(herr), hipMemcpyDeviceToHost, strm));
    HIP_CHECK(hipStreamSynchronize(strm));
    if (herr) throw std::invalid_argument("lsq_set_matrix_stencil: " + std::to_string(herr) +
                                          " nonzero entries fall outside [0, n_full)");
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
    S.has_var = false;
    for (int s = 0; s < n_stencil; ++s) {
        GenSt& G = h.st[s];
        G.grid = st[s].grid;
        G.ntpl = st[s].ntpl;
        G.row0 = st[s].row0;
        G.n_eq = st[s].n_eq;
        for (int d = 0; d < 3; ++d) {
            G.lo[d] = st[s].lo[d];
            G.hi[d] = st[s].hi[d];
        }
        G.F = nullptr;
        if (G.ntpl >= 1 && G.ntpl <= 8)
            for (int t = 0; t < G.ntpl; ++t) {
                for (int d = 0; d < 3; ++d) G.off[t][d] = st[s].off[t][d];
                G.val[t] = st[s].val[t];
                G.fsel[t] = 0;
            }
        for (const auto& f : S.sfields) {   // field-valued override (lsq_set_stencil_fields)
            if (f.stencil != s) continue;
            if (f.F.n < (int64_t)f.nfield * G.n_eq) throw std::invalid_argument("stencil fields: F too short");
            G.ntpl = f.ntpl;
            for (int t = 0; t < f.ntpl; ++t) {
                for (int d = 0; d < 3; ++d) G.off[t][d] = f.off[t][d];
                G.val[t] = f.val[t];
                G.fsel[t] = f.fsel[t];
            }
            G.F = G.n_eq ? f.F.p : nullptr;
            S.has_var = S.has_var || G.F;
        }
        if (G.grid < 0 || G.grid >= n_grids || G.ntpl < 1 || G.ntpl > (G.F ? MF_MAXT : 8))
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
    S.n_sorted_rows = npts;   // data rows: point order is random in space
    S.mf = !S.dist && describe_stencil_operator(S.mfh, m, n_full, n_grids, grids, npts, n_stencil, h.st);
    if (S.has_var && !S.mf)
        throw std::invalid_argument("lsq_set_matrix_stencil: field-valued parts need the structured operator "
                                    "(single GPU, parts inside their grids, |offsets| <= 3)");
    // structured single-GPU systems store only the data rows (System::g_full; LSQ_FULL_CSR=1 forms
    // everything up front, for A/B)
    static const bool full_env = getenv("LSQ_FULL_CSR") && getenv("LSQ_FULL_CSR")[0] == '1';
    const bool lazy = S.mf && !full_env;
    DBuf<double> dy(std::max<int64_t>(npts, 1)), dx(std::max<int64_t>(npts, 1)), dt;
    dy.upload(py, npts, strm);
    dx.upload(px, npts, strm);
    if (need_t) {
        dt.alloc(std::max<int64_t>(npts, 1));
        dt.upload(pt, npts, strm);
    }
    S.G = Csr{};
    S.GT = Csr{};
    S.gen_ctx.assign(reinterpret_cast<const char*>(&h), reinterpret_cast<const char*>(&h) + sizeof(GenCtx));
    S.g_full = true;
    gen_rows_csr(S, dy.p, dx.p, need_t ? dt.p : nullptr, lazy ? npts : m);
    if (lazy) {   // kept for ensure_full_csr
        S.gen_py = std::move(dy);
        S.gen_px = std::move(dx);
        S.gen_pt = std::move(dt);
        S.g_full = false;
    } else {
        S.gen_ctx.clear();
    }
    finish_formation(S);
    if (S.mf) build_dmf(S, n_grids, grids, n_interp, interp_grid, npts, py, px, pt);
}

void ensure_full_csr(System& S) {
    if (S.g_full) return;
    graph_cache_drop(&S);   // G is reallocated (a captured batch may hold the data-row CSR's pointers)
    gen_rows_csr(S, S.gen_py.p, S.gen_px.p, S.gen_pt.n ? S.gen_pt.p : nullptr, S.G.m);
    S.g_full = true;
    // the generation context stays (24 B per data row) so release_full_csr can drop G / GT again
    full_transpose(S);
}

bool release_full_csr(System& S) {
    if (!S.g_full || S.gen_ctx.empty() || S.dist) return false;   // nothing formed lazily, or relabelled
    graph_cache_drop(&S);
    S.sell_built = false;
    S.A = Sell();
    S.AT = Sell();
    S.GT = Csr{};
    S.G = Csr{};
    gen_rows_csr(S, S.gen_py.p, S.gen_px.p, S.gen_pt.n ? S.gen_pt.p : nullptr, S.mfh.npts);   // data rows only
    S.g_full = false;
    S.cs_mode = -1;   // the SELL values are gone; the next refresh fills the data rows' copies again
    S.iter_ready = false;
    return true;
}

int64_t stored_rows(const System& S) { return S.g_full ? S.G.m : S.mfh.npts; }

// Kept rows and their entries of the formed operator (lsq_shape).  A lazily formed system is not
// formed for it: the row generator's count pass runs again over every row, reduced on the device
// against the row mask (shape() used to form and keep the full G / GT).
void shape_counts(System& S, int64_t* mk, int64_t* zk) {
    hipStream_t strm = S.stream;
    const int64_t m = S.G.m;
    if (S.g_full) {
        std::vector<int64_t> rp(m + 1);
        std::vector<uint8_t> keep(m);
        S.G.rp.download(rp.data(), m + 1, strm);
        S.rowkeep.download(keep.data(), m, strm);
        HIP_CHECK(hipStreamSynchronize(strm));
        int64_t a = 0, z = 0;
        for (int64_t i = 0; i < m; ++i)
            if (keep[i]) { ++a; z += rp[i + 1] - rp[i]; }
        *mk = a;
        *zk = z;
        return;
    }
    const GenCtx& h = *reinterpret_cast<const GenCtx*>(S.gen_ctx.data());
    DBuf<GenCtx> dctx(1);
    HIP_CHECK(hipMemcpyAsync(dctx.p, &h, sizeof(GenCtx), hipMemcpyHostToDevice, strm));
    DBuf<unsigned long long> err(1), ks(2);
    err.zero(strm);
    ks.zero(strm);
    const int32_t* cmap = S.have_colmap ? S.colmap.p : nullptr;
    hipLaunchKernelGGL(k_gen_rows, dim3(grid_for(m)), dim3(BLOCK), 0, strm, 0, dctx.p, S.gen_py.p, S.gen_px.p,
                       S.gen_pt.n ? S.gen_pt.p : nullptr, cmap, nullptr, nullptr, nullptr, nullptr, err.p, m,
                       S.rowkeep.p, ks.p);
    KERNEL_CHECK();
    unsigned long long v[2] = {0, 0};
    ks.download(v, 2, strm);
    HIP_CHECK(hipStreamSynchronize(strm));
    *mk = (int64_t)v[0];
    *zk = (int64_t)v[1];
}

// z0 (gz) on a 2× refinement of the dz (g3) lattice: the points sorted by dz cell with their dz
// subscripts — the data rows of the system Galerkin-projected onto the dz lattice (z0's bilinear
// interpolation composed with the bilinear prolongation is the dz-lattice interpolation), the
// multigrid's level 1 (mg.inc mg_build_mixed).  Held by S.mx (column layout: z0 then dz).
void build_dmf_mixed(System& S, const lsq_grid_desc& gz, const lsq_grid_desc& g3, int64_t npts, const double* py,
                     const double* px, const double* pt) {
    DmfDesc D{};
    D.S0 = (int32_t)g3.shape[0];
    D.S1 = (int32_t)g3.shape[1];
    D.S2 = (int32_t)g3.shape[2];
    if (D.S0 < 2 || D.S1 < 2 || (int64_t)D.S0 * D.S1 * (1 + D.S2) >= (int64_t(1) << 31)) return;
    D.n2 = 1;
    D.col2[0] = 0;
    D.n3 = 1;
    D.col3 = (int64_t)D.S0 * D.S1;
    D.npts = npts;
    const int64_t C1 = D.S1 - 1, ncell = (int64_t)(D.S0 - 1) * C1;
    auto cell = [](double f, int S) {
        const int c = (int)std::floor(f);
        return std::min(std::max(c, 0), S - 2);
    };
    std::vector<double> F(3 * npts);
    std::vector<int64_t> key(npts);
    std::vector<int32_t> cnt(ncell + 1, 0);
    for (int64_t r = 0; r < npts; ++r) {
        const double fy = (py[r] - g3.b0[0]) / g3.delta[0], fx = (px[r] - g3.b0[1]) / g3.delta[1];
        const double ft = (pt[r] - g3.b0[2]) / g3.delta[2];
        if (!(fy >= 0.0 && fy <= D.S0 - 1 && fx >= 0.0 && fx <= D.S1 - 1 && ft >= 0.0 && ft <= D.S2 - 1)) return;
        F[3 * r] = fy;
        F[3 * r + 1] = fx;
        F[3 * r + 2] = ft;
        key[r] = (int64_t)cell(fy, D.S0) * C1 + cell(fx, D.S1);
        ++cnt[key[r] + 1];
    }
    for (int64_t c = 0; c < ncell; ++c) cnt[c + 1] += cnt[c];
    std::vector<int32_t> perm(npts), slot(cnt.begin(), cnt.end() - 1);
    std::vector<double> P(4 * npts);
    for (int64_t r = 0; r < npts; ++r) {
        const int32_t i = slot[key[r]]++;
        perm[i] = (int32_t)r;
        P[4 * i] = F[3 * r];
        P[4 * i + 1] = F[3 * r + 1];
        P[4 * i + 2] = F[3 * r + 2];
        P[4 * i + 3] = 1.0;
    }
    auto* X = new System();
    X->device = S.device;
    X->stream = S.stream;
    X->own_stream = false;
    X->dmf_pt.alloc(4 * npts);
    X->dmf_pt.upload(P.data(), 4 * npts, S.stream);
    X->dmf_perm.alloc(npts);
    X->dmf_perm.upload(perm.data(), npts, S.stream);
    X->dmf_cell.alloc(ncell + 1);
    X->dmf_cell.upload(cnt.data(), ncell + 1, S.stream);
    HIP_CHECK(hipStreamSynchronize(S.stream));
    D.ok = 1;
    X->dmf = D;
    X->mfh.npts = npts;
    S.mx = X;
    S.mx_z0col = (int32_t)gz.col0;
    S.mx_dzcol = (int32_t)g3.col0;
    S.mx_Sf0 = (int32_t)gz.shape[0];
    S.mx_Sf1 = (int32_t)gz.shape[1];
    S.mx_Sc0 = D.S0;
    S.mx_Sc1 = D.S1;
    S.mx_nt = D.S2;
}

// Matrix-free CGNR data rows (DmfDesc): eligible when every interpolation grid is 2-D or 3-D on one
// shared (y, x) lattice (≤ 2 2-D parts, ≤ 1 3-D part with ≤ CG_MAXT t nodes).  The float
// subscripts are computed here exactly as k_gen_rows computes them (one IEEE division each), the
// points counting-sorted by (y, x) cell (stable: data-row order within a cell).
void build_dmf(System& S, int32_t n_grids, const lsq_grid_desc* grids, int32_t n_interp, const int32_t* interp_grid,
               int64_t npts, const double* py, const double* px, const double* pt) {
    S.dmf = DmfDesc{};
    delete S.mx;
    S.mx = nullptr;
    if (const char* e = getenv("LSQ_CG_DMF"))
        if (e[0] == '0') return;
    if (n_interp < 1 || npts < 1 || npts >= (int64_t(1) << 31)) return;
    const lsq_grid_desc& g0 = grids[interp_grid[0]];
    DmfDesc D{};
    const lsq_grid_desc* g3 = nullptr;
    bool shared = true;
    for (int k = 0; k < n_interp; ++k) {
        const lsq_grid_desc& g = grids[interp_grid[k]];
        if (g.ndim < 2 || g.ndim > 3) return;
        for (int d = 0; d < 2; ++d)
            if (g.shape[d] != g0.shape[d] || g.b0[d] != g0.b0[d] || g.delta[d] != g0.delta[d]) shared = false;
        if (g.ndim == 2) {
            if (D.n2 == 2) return;
            D.col2[D.n2++] = g.col0;
        } else {
            if (D.n3 == 1 || g.shape[2] < 2 || g.shape[2] > CG_MAXT) return;
            D.col3 = g.col0;
            D.n3 = 1;
            g3 = &g;
        }
    }
    if (!shared) {   // z0 on a 2× refinement of the dz lattice: the multigrid's coarse data rows
        if (n_interp != 2 || D.n2 != 1 || D.n3 != 1) return;
        const lsq_grid_desc& gz = grids[interp_grid[0]].ndim == 2 ? grids[interp_grid[0]] : grids[interp_grid[1]];
        for (int d = 0; d < 2; ++d)
            if (gz.shape[d] != 2 * g3->shape[d] - 1 || gz.b0[d] != g3->b0[d] || 2.0 * gz.delta[d] != g3->delta[d]) return;
        build_dmf_mixed(S, gz, *g3, npts, py, px, pt);
        return;
    }
    if (g0.shape[0] < 2 || g0.shape[1] < 2 || (int64_t)g0.shape[0] * g0.shape[1] >= (int64_t(1) << 31)) return;
    D.S0 = (int32_t)g0.shape[0];
    D.S1 = (int32_t)g0.shape[1];
    D.S2 = g3 ? (int32_t)g3->shape[2] : 1;
    D.npts = npts;
    const int64_t C1 = D.S1 - 1, ncell = (int64_t)(D.S0 - 1) * C1;
    auto cell = [](double f, int S) {   // as the kernels: floor, clamped to the last cell
        const int c = (int)std::floor(f);
        return std::min(std::max(c, 0), S - 2);
    };
    std::vector<double> F(3 * npts);
    std::vector<int64_t> key(npts);
    std::vector<int32_t> cnt(ncell + 1, 0);
    for (int64_t r = 0; r < npts; ++r) {
        const double fy = (py[r] - g0.b0[0]) / g0.delta[0], fx = (px[r] - g0.b0[1]) / g0.delta[1];
        const double ft = g3 ? (pt[r] - g3->b0[2]) / g3->delta[2] : 0.0;
        if (!(fy >= 0.0 && fy <= D.S0 - 1 && fx >= 0.0 && fx <= D.S1 - 1)) return;   // formation rejected it
        if (g3 && !(ft >= 0.0 && ft <= D.S2 - 1)) return;
        F[3 * r] = fy;
        F[3 * r + 1] = fx;
        F[3 * r + 2] = ft;
        key[r] = (int64_t)cell(fy, D.S0) * C1 + cell(fx, D.S1);
        ++cnt[key[r] + 1];
    }
    for (int64_t c = 0; c < ncell; ++c) cnt[c + 1] += cnt[c];
    std::vector<int32_t> perm(npts), slot(cnt.begin(), cnt.end() - 1);
    std::vector<double> P(4 * npts);
    for (int64_t r = 0; r < npts; ++r) {
        const int32_t i = slot[key[r]]++;
        perm[i] = (int32_t)r;
        P[4 * i] = F[3 * r];
        P[4 * i + 1] = F[3 * r + 1];
        P[4 * i + 2] = F[3 * r + 2];
        P[4 * i + 3] = 1.0;   // row scale, refreshed per solve (cg_dmf_prepare)
    }
    S.dmf_pt.alloc(4 * npts);
    S.dmf_pt.upload(P.data(), 4 * npts, S.stream);
    S.dmf_perm.alloc(npts);
    S.dmf_perm.upload(perm.data(), npts, S.stream);
    S.dmf_cell.alloc(ncell + 1);
    S.dmf_cell.upload(cnt.data(), ncell + 1, S.stream);
    HIP_CHECK(hipStreamSynchronize(S.stream));
    D.ok = 1;
    S.dmf = D;
}

}  // namespace lsq
