// block.hip — block-Jacobi preconditioner (precond 3; SURVEY.md §8 a7.4 — the reference solves
// directly with SuiteSparseQR and has no counterpart).
//
// Right preconditioner M = blockdiag(R_b⁻¹) with R_bᵀR_b = (AᵀA)_bb, A = diag(rs)·G: LSQR runs on
// A·M, whose column blocks are orthonormal in the block's own metric.  For smooth_fit a block is
// one (y, x) node — its z0 column and the dz columns of every kept epoch — so the strong
// z0/dz/epoch coupling of the data rows and the time-derivative constraints is removed exactly;
// the iteration count then depends on the spatial coupling only.
//
// Factorisation: (AᵀA)_bb with one thread per (block, entry) — a merge of two sorted GT rows
// (deterministic, no atomics) — then one thread per block for the Cholesky and the triangular
// inverse, in place.  Columns
// whose pivot vanishes (empty or dependent inside the block) are dropped: their rows and columns
// of R_b⁻¹ are zero, so the iteration never moves them (x_j = 0).
#include <algorithm>
#include <vector>

#include "system.hpp"

namespace lsq {
namespace {

constexpr int KB = 16;                     // maximum block size
constexpr int KB_PACK = KB * (KB + 1) / 2;

__device__ __forceinline__ int pk(int i, int j) { return j * (j + 1) / 2 + i; }   // i <= j

// Σ_r rs_r² · G_ri · G_rj over the common rows of GT rows a and b (ascending row ids)
__device__ double col_dot(const int64_t* __restrict__ trp, const int32_t* __restrict__ tci,
                          const double* __restrict__ tval, const double* __restrict__ rs, int32_t a, int32_t b) {
    int64_t p = trp[a], pe = trp[a + 1], q = trp[b], qe = trp[b + 1];
    double s = 0.0;
    while (p < pe && q < qe) {
        const int32_t rp = tci[p], rq = tci[q];
        if (rp == rq) {
            const double w = rs[rp];
            s += (w * tval[p]) * (w * tval[q]);
            ++p;
            ++q;
        } else if (rp < rq) {
            ++p;
        } else {
            ++q;
        }
    }
    return s;
}

// (AᵀA)_bb, one thread per (block, packed entry): Ri[b·npk + e] ← N_ij (e = j(j+1)/2 + i)
__global__ __launch_bounds__(BLOCK) void k_block_normal(int64_t nb, int kmax, const int64_t* __restrict__ ptr,
                                                        const int32_t* __restrict__ cols,
                                                        const int64_t* __restrict__ trp,
                                                        const int32_t* __restrict__ tci,
                                                        const double* __restrict__ tval,
                                                        const double* __restrict__ rs, double* __restrict__ N) {
    const int npk = kmax * (kmax + 1) / 2;
    const int64_t total = nb * npk;
    for (int64_t q = (int64_t)blockIdx.x * BLOCK + threadIdx.x; q < total; q += (int64_t)gridDim.x * BLOCK) {
        const int64_t b = q / npk;
        const int e = (int)(q - b * npk);
        int j = 0;
        while ((j + 1) * (j + 2) / 2 <= e) ++j;
        const int i = e - j * (j + 1) / 2;
        const int64_t b0 = ptr[b];
        const int k = (int)(ptr[b + 1] - b0);
        N[q] = j < k ? col_dot(trp, tci, tval, rs, cols[b0 + i], cols[b0 + j]) : 0.0;
    }
}

// (AᵀA)_bb of a lazily formed structured system (System::g_full = false: no GT): the data rows by
// the merge over GdT (their transpose, rows = compact columns) and the stencil rows from the part
// descriptors — for columns i, j of one grid, Σ over the parts' rows that hold both: a row of
// centre c = sub(i) − off_t holds j when c + off_t2 = sub(j).  Same products as the GT merge.
__global__ __launch_bounds__(BLOCK) void k_block_normal_mf(int64_t nb, int kmax, const int64_t* __restrict__ ptr,
                                                           const int32_t* __restrict__ cols,
                                                           const int32_t* __restrict__ full,
                                                           const int64_t* __restrict__ trp,
                                                           const int32_t* __restrict__ tci,
                                                           const double* __restrict__ tval,
                                                           const MfDesc* __restrict__ dd,
                                                           const double* __restrict__ rs, double* __restrict__ N) {
    const MfDesc& d = *dd;
    const int npk = kmax * (kmax + 1) / 2;
    const int64_t total = nb * npk;
    for (int64_t q = (int64_t)blockIdx.x * BLOCK + threadIdx.x; q < total; q += (int64_t)gridDim.x * BLOCK) {
        const int64_t b = q / npk;
        const int e = (int)(q - b * npk);
        int j = 0;
        while ((j + 1) * (j + 2) / 2 <= e) ++j;
        const int i = e - j * (j + 1) / 2;
        const int64_t b0 = ptr[b];
        const int k = (int)(ptr[b + 1] - b0);
        if (j >= k) {
            N[q] = 0.0;
            continue;
        }
        double s = col_dot(trp, tci, tval, rs, cols[b0 + i], cols[b0 + j]);
        const int64_t fi = full[b0 + i], fj = full[b0 + j];
        for (int g = 0; g < d.n_grids; ++g) {
            const MfGrid& G = d.g[g];
            if (!G.nparts || fi < G.col0 || fi >= (int64_t)G.col0 + G.nodes) continue;
            if (fj < G.col0 || fj >= (int64_t)G.col0 + G.nodes) break;
            const int nd = G.ndim;
            int64_t si[3] = {0, 0, 0}, sj[3] = {0, 0, 0};
            int64_t ri = fi - G.col0, rj = fj - G.col0;
            for (int a = nd - 1; a >= 0; --a) {
                si[a] = ri % G.shape[a];
                ri /= G.shape[a];
                sj[a] = rj % G.shape[a];
                rj /= G.shape[a];
            }
            for (int pp = 0; pp < G.nparts; ++pp) {
                const MfPart& P = d.p[G.part[pp]];
                for (int t = 0; t < P.ntpl; ++t) {
                    int64_t kk = 0;
                    bool in = true;
                    for (int a = 0; a < nd; ++a) {
                        const int64_t c = si[a] - P.off[t][a];
                        in = in && c >= P.lo[a] && c < P.hi[a];
                        kk = kk * (P.hi[a] - P.lo[a]) + (c - P.lo[a]);
                    }
                    if (!in) continue;
                    const double w = rs[P.row0 + kk];
                    const double vi = P.var ? P.val[t] * P.F[(int64_t)P.fsel[t] * P.n_eq + kk] : P.val[t];
                    for (int t2 = 0; t2 < P.ntpl; ++t2) {
                        bool hit = true;
                        for (int a = 0; a < nd; ++a) hit = hit && si[a] - P.off[t][a] + P.off[t2][a] == sj[a];
                        if (!hit) continue;
                        const double vj = P.var ? P.val[t2] * P.F[(int64_t)P.fsel[t2] * P.n_eq + kk] : P.val[t2];
                        s += (w * vi) * (w * vj);
                    }
                }
            }
            break;
        }
        N[q] = s;
    }
}

// The same (AᵀA)_bb when every stencil part of the system has one row scale and constant
// coefficients (smooth_fit's constraints): a node column's own entries of the stencil part depend
// on the node only through its boundary class (as the CG's normal-stencil tables,
// ns_from_parts in lsqr_cg.inc), so the part loop above — 64-bit index arithmetic and a
// template-pair search per entry, 54 ms at C4 — becomes one table read per entry.  Table of grid
// g: coef[coef0 + ((cy·ncls1 + cx)·ncls2 + ct)·BN_NDT + dt + BN_DT] (dt = t_j − t_i; the rows of
// the class representative, summed in ns_from_parts' order: parts, t1, t2).
constexpr int BN_DT = KB - 1, BN_NDT = 2 * BN_DT + 1;
struct BnGrid {
    int32_t col0, nodes, S[3], K[3], ncls[3], coef0;
    FastDiv fd1, fd2;   // by shape[1] · shape[2] and by shape[2]
};
struct BnDesc {
    int32_t n;
    BnGrid g[MF_MAX_GRIDS];
};
__device__ __forceinline__ uint32_t bn_div(uint32_t n, const FastDiv& f) {
    return (uint32_t)(((uint64_t)n * f.mul) >> (32 + f.shift));
}
__device__ __forceinline__ int bn_cls(int c, int n, int K, int ncls) {
    return ncls == n ? c : (c < K ? c : (c >= n - K ? c - n + 2 * K + 1 : K));
}
__global__ __launch_bounds__(BLOCK) void k_block_normal_tab(int64_t nb, int kmax, const int64_t* __restrict__ ptr,
                                                            const int32_t* __restrict__ cols,
                                                            const int32_t* __restrict__ full,
                                                            const int64_t* __restrict__ trp,
                                                            const int32_t* __restrict__ tci,
                                                            const double* __restrict__ tval,
                                                            const double* __restrict__ rs, BnDesc D,
                                                            const double* __restrict__ coef, double* __restrict__ N,
                                                            int* __restrict__ cross) {
    const int npk = kmax * (kmax + 1) / 2;
    const int64_t total = nb * npk;
    for (int64_t q = (int64_t)blockIdx.x * BLOCK + threadIdx.x; q < total; q += (int64_t)gridDim.x * BLOCK) {
        const int64_t b = q / npk;
        const int e = (int)(q - b * npk);
        int j = 0;
        while ((j + 1) * (j + 2) / 2 <= e) ++j;
        const int i = e - j * (j + 1) / 2;
        const int64_t b0 = ptr[b];
        const int k = (int)(ptr[b + 1] - b0);
        if (j >= k) {
            N[q] = 0.0;
            continue;
        }
        double s = col_dot(trp, tci, tval, rs, cols[b0 + i], cols[b0 + j]);
        const int fi = full[b0 + i], fj = full[b0 + j];
        for (int g = 0; g < D.n; ++g) {
            const BnGrid& G = D.g[g];
            if (fi < G.col0 || fi >= G.col0 + G.nodes) continue;
            if (fj < G.col0 || fj >= G.col0 + G.nodes) break;
            const uint32_t ri = (uint32_t)(fi - G.col0), rj = (uint32_t)(fj - G.col0);
            const uint32_t ni = bn_div(ri, G.fd2), nj = bn_div(rj, G.fd2);   // (y, x) node
            if (ni != nj) {   // a block spanning two nodes of one grid: the tables miss their coupling
                atomicOr(cross, 1);
                break;
            }
            const int ti = (int)(ri - ni * (uint32_t)G.S[2]), dt = (int)(rj - nj * (uint32_t)G.S[2]) - ti;
            const uint32_t y = bn_div(ri, G.fd1);
            const int x = (int)(ni - y * (uint32_t)G.S[1]);
            const int cy = bn_cls((int)y, G.S[0], G.K[0], G.ncls[0]), cx = bn_cls(x, G.S[1], G.K[1], G.ncls[1]);
            const int ct = bn_cls(ti, G.S[2], G.K[2], G.ncls[2]);
            if (dt >= -BN_DT && dt <= BN_DT)
                s += coef[G.coef0 + ((cy * G.ncls[1] + cx) * G.ncls[2] + ct) * BN_NDT + dt + BN_DT];
            break;
        }
        N[q] = s;
    }
}

// Host: the tables of k_block_normal_tab from the part descriptors; false when a part has per-row
// scales or field-valued coefficients (then k_block_normal_mf)
static int bn_rep(int k, int n, int K, int ncls) { return ncls == n ? k : (k <= K ? k : n - 2 * K - 1 + k); }
bool block_normal_tables(const MfDesc& d, BnDesc& D, std::vector<double>& coef) {
    D = BnDesc{};
    coef.clear();
    D.n = d.n_grids;
    for (int g = 0; g < d.n_grids; ++g) {
        const MfGrid& G = d.g[g];
        BnGrid& B = D.g[g];
        B.col0 = G.col0;
        B.nodes = G.nparts ? G.nodes : 0;   // grids without parts: no stencil entries
        for (int e = 0; e < 3; ++e) B.S[e] = G.ndim > e ? G.shape[e] : 1;
        int K[3] = {0, 0, 0};
        for (int qq = 0; qq < G.nparts; ++qq) {
            const MfPart& P = d.p[G.part[qq]];
            if (!P.wconst || P.var) return false;
            for (int e = 0; e < 3; ++e) {
                int omin = 1 << 20, omax = -(1 << 20);
                for (int t = 0; t < P.ntpl; ++t) {
                    omin = std::min(omin, P.off[t][e]);
                    omax = std::max(omax, P.off[t][e]);
                }
                K[e] = std::max({K[e], P.lo[e] + omax, B.S[e] - P.hi[e] - omin, 0});
            }
        }
        for (int e = 0; e < 3; ++e) {
            B.K[e] = K[e];
            B.ncls[e] = B.S[e] <= 2 * K[e] + 1 ? B.S[e] : 2 * K[e] + 1;
        }
        B.fd1 = make_fastdiv((uint32_t)B.S[1] * (uint32_t)B.S[2]);
        B.fd2 = make_fastdiv((uint32_t)B.S[2]);
        B.coef0 = (int32_t)coef.size();
        if (!G.nparts) continue;
        coef.resize(coef.size() + (size_t)B.ncls[0] * B.ncls[1] * B.ncls[2] * BN_NDT, 0.0);
        for (int cy = 0; cy < B.ncls[0]; ++cy)
            for (int cx = 0; cx < B.ncls[1]; ++cx)
                for (int ct = 0; ct < B.ncls[2]; ++ct) {
                    const int pos[3] = {bn_rep(cy, B.S[0], K[0], B.ncls[0]), bn_rep(cx, B.S[1], K[1], B.ncls[1]),
                                        bn_rep(ct, B.S[2], K[2], B.ncls[2])};
                    double* row = coef.data() + B.coef0 + ((size_t)(cy * B.ncls[1] + cx) * B.ncls[2] + ct) * BN_NDT;
                    for (int qq = 0; qq < G.nparts; ++qq) {
                        const MfPart& P = d.p[G.part[qq]];
                        for (int t1 = 0; t1 < P.ntpl; ++t1) {
                            bool in = true;   // the row centred at pos − o_t1 exists
                            for (int e = 0; e < 3; ++e) {
                                const int ce = pos[e] - P.off[t1][e];
                                in = in && ce >= P.lo[e] && ce < P.hi[e];
                            }
                            if (!in) continue;
                            for (int t2 = 0; t2 < P.ntpl; ++t2) {
                                if (P.off[t2][0] != P.off[t1][0] || P.off[t2][1] != P.off[t1][1]) continue;
                                const int dt = P.off[t2][2] - P.off[t1][2];
                                if (dt < -BN_DT || dt > BN_DT) continue;   // beyond any block
                                row[dt + BN_DT] += (P.w * P.val[t1]) * (P.w * P.val[t2]);
                            }
                        }
                    }
                }
    }
    return true;
}

// In place: N_b -> R_b (Cholesky, upper) -> R_b⁻¹, one thread per block
__global__ __launch_bounds__(BLOCK) void k_block_factor(int64_t nb, const int64_t* __restrict__ ptr, int kmax,
                                                        double* __restrict__ Ri, unsigned long long* ndead) {
    const int npk = kmax * (kmax + 1) / 2;
    for (int64_t b = (int64_t)blockIdx.x * BLOCK + threadIdx.x; b < nb; b += (int64_t)gridDim.x * BLOCK) {
        const int k = (int)(ptr[b + 1] - ptr[b]);
        double R[KB_PACK];   // N, then R in place (upper, packed by columns)
        double d0[KB];
        for (int e = 0; e < k * (k + 1) / 2; ++e) R[e] = Ri[b * npk + e];
        for (int j = 0; j < k; ++j) d0[j] = R[pk(j, j)];
        bool dead[KB];
        // Cholesky by columns: R_ij = (N_ij − Σ_{l<i} R_li R_lj) / R_ii, R_jj = sqrt(N_jj − Σ R_lj²)
        for (int j = 0; j < k; ++j) {
            for (int i = 0; i < j; ++i) {
                if (dead[i]) {
                    R[pk(i, j)] = 0.0;
                    continue;
                }
                double s = R[pk(i, j)];
                for (int l = 0; l < i; ++l) s -= R[pk(l, i)] * R[pk(l, j)];
                R[pk(i, j)] = s / R[pk(i, i)];
            }
            double d = R[pk(j, j)];
            for (int l = 0; l < j; ++l) d -= R[pk(l, j)] * R[pk(l, j)];
            dead[j] = !(d > 1e-12 * d0[j]) || !(d0[j] > 0.0);
            if (dead[j]) {
                for (int l = 0; l < j; ++l) R[pk(l, j)] = 0.0;
                R[pk(j, j)] = 1.0;
                atomicAdd(ndead, 1ull);
            } else {
                R[pk(j, j)] = sqrt(d);
            }
        }
        // R⁻¹ (upper) column by column from the diagonal up
        double X[KB_PACK];
        for (int j = 0; j < k; ++j) {
            X[pk(j, j)] = 1.0 / R[pk(j, j)];
            for (int i = j - 1; i >= 0; --i) {
                double s = 0.0;
                for (int l = i + 1; l <= j; ++l) s += R[pk(i, l)] * X[pk(l, j)];
                X[pk(i, j)] = -s / R[pk(i, i)];
            }
        }
        for (int j = 0; j < k; ++j)
            for (int i = 0; i <= j; ++i)
                if (dead[i] || dead[j]) X[pk(i, j)] = 0.0;
        for (int e = 0; e < npk; ++e) Ri[b * npk + e] = e < k * (k + 1) / 2 ? X[e] : 0.0;
    }
}

// The same for blocks of exactly K columns (smooth_fit's node blocks, the multigrid levels' blocks):
// the block lives in registers (fully unrolled, compile-time indices) instead of the generic
// kernel's scratch arrays — that kernel's thread walks ~2 000 dependent scratch accesses, 150 µs
// even for a level of 256 blocks.  R⁻¹ overwrites R in place, columns right to left and rows
// bottom-up (X_ij needs R's row i right of i only in columns ≤ j, still R, and X_lj, l > i, already
// written): the same expressions in the same order as k_block_factor, so the same values.
template <int K>
__global__ __launch_bounds__(BLOCK) void k_block_factor_k(int64_t nb, double* __restrict__ Ri,
                                                          unsigned long long* ndead) {
    constexpr int NP = K * (K + 1) / 2;
    for (int64_t b = (int64_t)blockIdx.x * BLOCK + threadIdx.x; b < nb; b += (int64_t)gridDim.x * BLOCK) {
        double R[NP];
        double* __restrict__ blk = Ri + b * NP;
#pragma unroll
        for (int e = 0; e < NP; ++e) R[e] = blk[e];
        double d0[K];
#pragma unroll
        for (int j = 0; j < K; ++j) d0[j] = R[pk(j, j)];
        unsigned dead = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
#pragma unroll
            for (int i = 0; i < j; ++i) {
                double s = R[pk(i, j)];
#pragma unroll
                for (int l = 0; l < i; ++l) s -= R[pk(l, i)] * R[pk(l, j)];
                R[pk(i, j)] = ((dead >> i) & 1u) ? 0.0 : s / R[pk(i, i)];
            }
            double d = R[pk(j, j)];
#pragma unroll
            for (int l = 0; l < j; ++l) d -= R[pk(l, j)] * R[pk(l, j)];
            const bool dj = !(d > 1e-12 * d0[j]) || !(d0[j] > 0.0);
            if (dj) {
                dead |= 1u << j;
                atomicAdd(ndead, 1ull);
            }
#pragma unroll
            for (int l = 0; l < j; ++l) R[pk(l, j)] = dj ? 0.0 : R[pk(l, j)];
            R[pk(j, j)] = dj ? 1.0 : sqrt(d);
        }
#pragma unroll
        for (int j = K - 1; j >= 0; --j) {
            const double rjj = R[pk(j, j)];
            R[pk(j, j)] = 1.0 / rjj;
#pragma unroll
            for (int i = j - 1; i >= 0; --i) {
                double s = 0.0;
#pragma unroll
                for (int l = i + 1; l <= j; ++l) s += R[pk(i, l)] * R[pk(l, j)];
                R[pk(i, j)] = -s / R[pk(i, i)];
            }
        }
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
            for (int i = 0; i <= j; ++i)
                if (((dead >> i) | (dead >> j)) & 1u) R[pk(i, j)] = 0.0;
#pragma unroll
        for (int e = 0; e < NP; ++e) blk[e] = R[e];
    }
}

// R_b⁻¹ rounded to fp32 for CG's z = R_b⁻¹(R_b⁻ᵀ s): packed upper, block stride npks (npk rounded
// up to even, so a run of blocks starts 8-byte aligned).  L L^T with a triangular L whose diagonal
// is non-zero stays SPD whatever the rounding, so CG keeps a valid preconditioner at half the bytes.
// Lf = R_b⁻¹ rounded to lf_t; round_ri: Ri takes the rounded values too, so every consumer of the
// system's block preconditioner (LSQR's epilogue from Lf, its x = M y and warm start from Ri, CGNR
// from Lf) applies one and the same M
__global__ __launch_bounds__(BLOCK) void k_block_rinv32(int64_t nb, int npk, int npks, double* __restrict__ Ri,
                                                        lf_t* __restrict__ Lf, int round_ri) {
    for (int64_t q = (int64_t)blockIdx.x * BLOCK + threadIdx.x; q < nb * npks; q += (int64_t)gridDim.x * BLOCK) {
        const int64_t b = q / npks;
        const int e = (int)(q - b * npks);
        const lf_t v = e < npk ? lf_round(Ri[b * npk + e]) : lf_t(0);
        Lf[q] = v;
        if (round_ri && e < npk) Ri[b * npk + e] = (double)lf_val(v);
    }
}

__global__ __launch_bounds__(BLOCK) void k_full_ids(int64_t n, const int32_t* __restrict__ cols,
                                                    const int32_t* __restrict__ keep, int32_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK)
        out[i] = keep ? keep[cols[i]] : cols[i];
}

// affine blocks: ptr[b] = b·k; column j of block b = base_j + b·stride_j (compact), checked: in
// range, each compact column in exactly one block (nb·k == n), full id fbase_j + b·fstride_j
struct AffDesc {
    int64_t base[KB], stride[KB], fbase[KB], fstride[KB];
};
__global__ __launch_bounds__(BLOCK) void k_affine_blocks(int64_t nb, int k, int64_t n, AffDesc a,
                                                         const int32_t* __restrict__ keep, int64_t* __restrict__ ptr,
                                                         int32_t* __restrict__ cols, int32_t* __restrict__ full,
                                                         int* __restrict__ seen, int* __restrict__ err) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < nb * k; i += (int64_t)gridDim.x * BLOCK) {
        const int64_t b = i / k;
        const int j = (int)(i - b * k);
        if (j == 0) ptr[b] = b * k;
        if (i == 0) ptr[nb] = nb * k;
        const int64_t c = a.base[j] + b * a.stride[j];
        if (c < 0 || c >= n) {
            atomicOr(err, 1);
            cols[i] = 0;
            full[i] = 0;
            continue;
        }
        cols[i] = (int32_t)c;
        const int64_t f = keep ? keep[c] : c;
        full[i] = (int32_t)f;
        if (f != a.fbase[j] + b * a.fstride[j]) atomicOr(err, 2);
        if (atomicAdd(seen + c, 1) != 0) atomicOr(err, 4);
    }
}

}  // namespace

// Column blocks given by their affine structure (lsq_set_column_blocks_affine): the arrays of
// set_column_blocks formed on the device, the structure checked there; no host column lists.
void set_column_blocks_affine(System& S, int64_t nb, int k, const int64_t* base, const int64_t* stride,
                              const int64_t* fbase, const int64_t* fstride) {
    const int64_t n = S.G.n;
    if (nb < 1 || k < 1 || k > KB || !base || !stride || !fbase || !fstride)
        throw std::invalid_argument("lsq_set_column_blocks_affine: bad arguments");
    if (nb * k != n) throw std::invalid_argument("lsq_set_column_blocks_affine: the blocks must cover every column");
    AffDesc a{};
    for (int j = 0; j < k; ++j) {
        a.base[j] = base[j];
        a.stride[j] = stride[j];
        a.fbase[j] = fbase[j];
        a.fstride[j] = fstride[j];
    }
    S.blk_ptr.alloc(nb + 1);
    S.blk_cols.alloc(n);
    S.blk_full.alloc(n);
    DBuf<int> seen(n), err(1);
    seen.zero(S.stream);
    err.zero(S.stream);
    hipLaunchKernelGGL(k_affine_blocks, dim3(grid_for(n)), dim3(BLOCK), 0, S.stream, nb, k, n, a,
                       S.mf ? S.keep.p : nullptr, S.blk_ptr.p, S.blk_cols.p, S.blk_full.p, seen.p, err.p);
    KERNEL_CHECK();
    int e = 0;
    err.download(&e, 1, S.stream);
    HIP_CHECK(hipStreamSynchronize(S.stream));
    if (e) {
        S.nblk = 0;   // no half-formed structure left behind (precond 3 then takes singletons)
        S.blk_kmax = 0;
        S.blk_affine = S.blk_user = S.blk_valid = false;
        S.blk_ptr = DBuf<int64_t>();
        S.blk_cols = DBuf<int32_t>();
        S.blk_full = DBuf<int32_t>();
        S.blk_Ri = DBuf<double>();
        S.iter_ready = false;
        throw std::invalid_argument(e & 1 ? "lsq_set_column_blocks_affine: column out of range"
                                    : e & 4 ? "lsq_set_column_blocks_affine: column in two blocks"
                                            : "lsq_set_column_blocks_affine: full column ids differ from full_base / full_stride");
    }
    S.nblk = nb;
    S.blk_kmax = k;
    S.blk_affine = nb > 1;
    for (int j = 0; j < k; ++j) {
        S.blk_aff.base[j] = fbase[j];
        S.blk_aff.stride[j] = fstride[j];
    }
    S.blk_Ri = DBuf<double>();
    S.blk_valid = false;
    S.blk_user = true;
    S.iter_ready = false;
}

void set_column_blocks(System& S, int64_t nb, const int64_t* ptr, const int32_t* cols) {
    const int64_t n = S.G.n;
    std::vector<int64_t> P;
    std::vector<int32_t> C;
    std::vector<uint8_t> seen(n, 0);
    P.reserve((size_t)std::max<int64_t>(nb, 0) + 1);
    C.reserve((size_t)n);
    P.push_back(0);
    int kmax = 1;
    if (nb > 0) {
        if (!ptr || !cols || ptr[0] != 0) throw std::invalid_argument("lsq_set_column_blocks: bad block_ptr");
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t k = ptr[b + 1] - ptr[b];
            if (k < 1 || k > KB) throw std::invalid_argument("lsq_set_column_blocks: block size must be 1..16");
            for (int64_t e = ptr[b]; e < ptr[b + 1]; ++e) {
                const int32_t c = cols[e];
                if (c < 0 || c >= n) throw std::invalid_argument("lsq_set_column_blocks: column out of range");
                if (seen[c]) throw std::invalid_argument("lsq_set_column_blocks: column in two blocks");
                seen[c] = 1;
                C.push_back(c);
            }
            P.push_back((int64_t)C.size());
            kmax = std::max<int>(kmax, (int)k);
        }
    }
    for (int64_t c = 0; c < n; ++c)   // the rest: singletons
        if (!seen[c]) {
            C.push_back((int32_t)c);
            P.push_back((int64_t)C.size());
        }
    S.nblk = (int64_t)P.size() - 1;
    S.blk_kmax = kmax;
    S.blk_ptr.alloc(S.nblk + 1);
    S.blk_ptr.upload(P.data(), S.nblk + 1, S.stream);
    S.blk_cols.alloc(std::max<int64_t>((int64_t)C.size(), 1));
    S.blk_cols.upload(C.data(), (int64_t)C.size(), S.stream);
    S.blk_full.alloc(std::max<int64_t>((int64_t)C.size(), 1));
    hipLaunchKernelGGL(k_full_ids, dim3(grid_for((int64_t)C.size())), dim3(BLOCK), 0, S.stream, (int64_t)C.size(),
                       S.blk_cols.p, S.mf ? S.keep.p : nullptr, S.blk_full.p);
    KERNEL_CHECK();
    // affine column ids (every block the same size, column j of block b at base_j + b·stride_j)
    S.blk_affine = false;
    if (S.nblk > 1 && (int64_t)C.size() == S.nblk * kmax) {
        std::vector<int32_t> F(C.size());
        S.blk_full.download(F.data(), (int64_t)C.size(), S.stream);
        HIP_CHECK(hipStreamSynchronize(S.stream));
        bool ok = true;
        for (int j = 0; j < kmax; ++j) {
            S.blk_aff.base[j] = F[j];
            S.blk_aff.stride[j] = (int64_t)F[kmax + j] - F[j];
        }
        for (int64_t b = 0; b < S.nblk && ok; ++b)
            for (int j = 0; j < kmax; ++j)
                ok = ok && (int64_t)F[b * kmax + j] == S.blk_aff.base[j] + b * S.blk_aff.stride[j];
        S.blk_affine = ok;
    }
    S.blk_Ri = DBuf<double>();
    S.blk_valid = false;
    S.blk_user = nb > 0;
    S.iter_ready = false;
    HIP_CHECK(hipStreamSynchronize(S.stream));
}

void ensure_blocks(System& S) {
    if (S.nblk == 0) set_column_blocks(S, 0, nullptr, nullptr);
}

// (AᵀA)_bb of every block into blk_Ri (packed upper), from the system's own rows
void block_normal(System& S) {
    ensure_blocks(S);
    const int npk = S.blk_kmax * (S.blk_kmax + 1) / 2;
    if (S.blk_Ri.n != (int64_t)npk * S.nblk) {
        graph_cache_drop(&S);   // captured block-preconditioned batches hold the old pointers
        S.blk_Ri.alloc((int64_t)npk * S.nblk);
    }
    BnDesc bd;
    std::vector<double> tab;
    const bool tab_env = !(getenv("LSQ_BLK_TAB") && getenv("LSQ_BLK_TAB")[0] == '0');   // A/B + parity test (per call)
    // lazily formed, class tables: they hold the stencil terms between columns of ONE (y, x) node
    // only, so a block that pairs two nodes of one grid (a user block set by lsq_set_column_blocks)
    // is flagged by the kernel and the block normals are redone by the part-descriptor kernel
    bool tab_done = false;
    if (!S.g_full && tab_env && block_normal_tables(S.mfh, bd, tab)) {
        S.blk_tab.alloc(std::max<int64_t>((int64_t)tab.size(), 1));
        S.blk_tab.upload(tab.data(), (int64_t)tab.size(), S.stream);
        DBuf<int> cross(1);
        cross.zero(S.stream);
        hipLaunchKernelGGL(k_block_normal_tab, dim3(grid_for(S.nblk * npk)), dim3(BLOCK), 0, S.stream, S.nblk,
                           S.blk_kmax, S.blk_ptr.p, S.blk_cols.p, S.blk_full.p, S.GdT.rp.p, S.GdT.ci.p, S.GdT.val.p,
                           S.rs.p, bd, S.blk_tab.p, S.blk_Ri.p, cross.p);
        KERNEL_CHECK();
        int c = 0;
        cross.download(&c, 1, S.stream);
        HIP_CHECK(hipStreamSynchronize(S.stream));
        tab_done = c == 0;
    }
    if (tab_done) {
    } else if (!S.g_full)   // lazily formed structured system: GdT + the stencil parts
        hipLaunchKernelGGL(k_block_normal_mf, dim3(grid_for(S.nblk * npk)), dim3(BLOCK), 0, S.stream, S.nblk,
                           S.blk_kmax, S.blk_ptr.p, S.blk_cols.p, S.blk_full.p, S.GdT.rp.p, S.GdT.ci.p, S.GdT.val.p,
                           S.mfd.p, S.rs.p, S.blk_Ri.p);
    else
        hipLaunchKernelGGL(k_block_normal, dim3(grid_for(S.nblk * npk)), dim3(BLOCK), 0, S.stream, S.nblk, S.blk_kmax,
                           S.blk_ptr.p, S.blk_cols.p, S.GT.rp.p, S.GT.ci.p, S.GT.val.p, S.rs.p, S.blk_Ri.p);
    KERNEL_CHECK();
}

// blk_Ri: (AᵀA)_bb -> R_b⁻¹ in place
void block_factor_in_place(System& S) {
    DBuf<unsigned long long> nd(1);
    nd.zero(S.stream);
    if (S.blk_affine && S.blk_kmax == 12)   // every block of 12 columns
        hipLaunchKernelGGL(k_block_factor_k<12>, dim3(grid_for(S.nblk)), dim3(BLOCK), 0, S.stream, S.nblk, S.blk_Ri.p,
                           nd.p);
    else
        hipLaunchKernelGGL(k_block_factor, dim3(grid_for(S.nblk)), dim3(BLOCK), 0, S.stream, S.nblk, S.blk_ptr.p,
                           S.blk_kmax, S.blk_Ri.p, nd.p);
    KERNEL_CHECK();
    const int npk = S.blk_kmax * (S.blk_kmax + 1) / 2, npks = lf_stride(npk);   // CGNR's copy
    if (S.blk_Lf.n != (int64_t)npks * S.nblk) {
        graph_cache_drop(&S);
        S.blk_Lf.alloc((int64_t)npks * S.nblk);
    }
    hipLaunchKernelGGL(k_block_rinv32, dim3(grid_for(S.nblk * npks)), dim3(BLOCK), 0, S.stream, S.nblk, npk, npks,
                       S.blk_Ri.p, S.blk_Lf.p, 1);
    KERNEL_CHECK();
    HIP_CHECK(hipStreamSynchronize(S.stream));
    S.blk_valid = true;
}

void block_factor(System& S) {
    block_normal(S);
    block_factor_in_place(S);
}

// Multigrid coarse levels (mg.inc): nb packed blocks (AᵀA)_bb of kmax columns in Ri -> R_b⁻¹ in
// place, then the fp32 copy Lf (block stride npks = npk rounded up to even).  ptr: device block
// pointers (b·kmax).  Asynchronous on `st`.
void block_factor_packed(int64_t nb, const int64_t* ptr, int kmax, double* Ri, lf_t* Lf,
                         unsigned long long* ndead, hipStream_t st) {
    if (kmax == 12)   // ptr = b·kmax: every block of kmax columns
        hipLaunchKernelGGL(k_block_factor_k<12>, dim3(grid_for(nb)), dim3(BLOCK), 0, st, nb, Ri, ndead);
    else
        hipLaunchKernelGGL(k_block_factor, dim3(grid_for(nb)), dim3(BLOCK), 0, st, nb, ptr, kmax, Ri, ndead);
    KERNEL_CHECK();
    const int npk = kmax * (kmax + 1) / 2, npks = lf_stride(npk);
    hipLaunchKernelGGL(k_block_rinv32, dim3(grid_for(nb * npks)), dim3(BLOCK), 0, st, nb, npk, npks, Ri, Lf, 0);
    KERNEL_CHECK();
}

}  // namespace lsq
