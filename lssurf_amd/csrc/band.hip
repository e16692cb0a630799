// band.hip — error propagation (smooth_fit compute_E, smooth_fit.py:212-274) without a dense
// factor.
//
// The reference factors A = Q R E' with SuiteSparseQR (`sparseqr.rz`, :218), inverts R column by
// column with the Cython `inv_tr_upper` (|x| > 1e-5 kept, :240-248) and reports
// E0 = sqrt(row sums of R⁻¹²) = sqrt(diag((AᵀA)⁻¹)) (:253) and, for every averaging operator,
// sqrt(row sums of (op·R⁻¹)²) = sqrt(diag(op (AᵀA)⁻¹ opᵀ)) (:266-270).  With the columns ordered
// so that AᵀA is banded — smooth_fit's columns node-major ((y, x) rows of nodes, each node's z0 and
// kept dz epochs together): a band of ~2 node rows — the factor is banded too:
//
//   N = AᵀA           in the caller's column order, stored as a band of 64×64 tiles (tile row I
//                     keeps tiles I..I+w, w from the row pattern of A), upper triangle, then
//                     equilibrated (S N S, S = diag(N)^-1/2)
//   N = RᵀR           right-looking tile Cholesky inside the band: per tile column K, POTRF of
//                     the diagonal tile (+ D_K = R_KK⁻¹), TRSM of the tile row by substitution,
//                     SYRK/GEMM of the trailing triangle on f64 MFMA
//   rows of R⁻¹       y = R⁻ᵀ e_j by banded forward sweeps, 64 right-hand sides per workgroup,
//                     Y_K = D_Kᵀ (O_K − Σ_{I=K−w}^{K−1} R_IKᵀ Y_I), only the last w+1 tiles of y
//                     live (a ring per workgroup); E_j² = ‖y‖²; op rows the same way with o = op_i
//
// Cost ~T²(w+1)/2 tile products (T = n/64) against the dense path's 2n³/3 flops (dense.hip), the
// same accuracy class as the dense R⁻¹ (measured 1e-13 relative to LAPACK at 48²×12), band
// storage n·(w+1)·64 doubles.  Takahashi's recurrence for the band of (AᵀA)⁻¹ costs only
// ~T(w+1)² but its sums cancel in proportion to cond(AᵀA): measured 3e-6 relative at 48²×12,
// 2 % at 64²×12 and negative diagonals beyond — so it is not used.
#include <chrono>
#include <algorithm>
#include <climits>
#include <memory>
#include <cmath>
#include <stdexcept>
#include <vector>

#include "system.hpp"

namespace lsq {
namespace {

constexpr int TB = 64;
constexpr int64_t TT = (int64_t)TB * TB;
constexpr int LDP = TB + 1;   // LDS tile pitch
typedef double d4 __attribute__((ext_vector_type(4)));

struct BandDev {
    int64_t T;    // tile rows (n padded to T·64)
    int w;        // tiles right of the diagonal kept per tile row
    double* R;    // Cholesky factor band
    double* D;    // R_KK⁻¹ per tile row
};

__device__ __forceinline__ double* btile(double* base, int w, int64_t I, int64_t J) {
    return base + ((I * (w + 1)) + (J - I)) * TT;
}

// LDS image of a row-major 64×64 tile (TR: transposed)
template <bool TR>
__device__ __forceinline__ void lds_tile(double* S, const double* __restrict__ src) {
    for (int idx = threadIdx.x; idx < TT; idx += BLOCK) {
        const int r = idx >> 6, c = idx & 63;
        const double v = src[idx];
        if (TR) S[c * LDP + r] = v;
        else S[r * LDP + c] = v;
    }
}

// acc += op(A)·B over one 64-deep tile pair held in LDS (A [i][k], or [k][i] when AT; B [k][j]);
// wave wv owns the 32×32 output block (r0, c0) as 2×2 f64 16×16x4 MFMA accumulators: element
// (s, t, reg) is row r0 + 16s + (lane>>4) + 4·reg, column c0 + 16t + (lane&15)
template <bool AT = false>
__device__ __forceinline__ void mma_tile(const double* A, const double* B, d4 (&acc)[2][2]) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r0 = (wv >> 1) * 32, c0 = (wv & 1) * 32;
    const int li = lane & 15, lk = lane >> 4;
#pragma unroll 4
    for (int k0 = 0; k0 < TB; k0 += 4) {
        const int k = k0 + lk;
        const double a0 = AT ? A[k * LDP + r0 + li] : A[(r0 + li) * LDP + k];
        const double a1 = AT ? A[k * LDP + r0 + 16 + li] : A[(r0 + 16 + li) * LDP + k];
        const double b0 = B[k * LDP + c0 + li], b1 = B[k * LDP + c0 + 16 + li];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
}

// a tile pair in registers (16-byte loads, 8 per thread per tile) and from there into LDS, so
// the next pair's loads are in flight while the MFMAs of the current one run
struct TilePair {
    double2 a[TT / 2 / BLOCK], b[TT / 2 / BLOCK];
    __device__ __forceinline__ void load(const double* __restrict__ pa, const double* __restrict__ pb) {
        const double2* a2 = reinterpret_cast<const double2*>(pa);
        const double2* b2 = reinterpret_cast<const double2*>(pb);
#pragma unroll
        for (int i = 0; i < TT / 2 / BLOCK; ++i) {
            a[i] = a2[threadIdx.x + BLOCK * i];
            b[i] = b2[threadIdx.x + BLOCK * i];
        }
    }
    __device__ __forceinline__ void store(double* SA, double* SB) const {
#pragma unroll
        for (int i = 0; i < TT / 2 / BLOCK; ++i) {
            const int idx = 2 * (threadIdx.x + BLOCK * i), r = idx >> 6, c = idx & 63;
            SA[r * LDP + c] = a[i].x;
            SA[r * LDP + c + 1] = a[i].y;
            SB[r * LDP + c] = b[i].x;
            SB[r * LDP + c + 1] = b[i].y;
        }
    }
};

__device__ __forceinline__ void acc_zero(d4 (&acc)[2][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[s][t] = d4{0.0, 0.0, 0.0, 0.0};
}

// visit every accumulator element: f(row, col, value&)
template <class F>
__device__ __forceinline__ void acc_each(d4 (&acc)[2][2], F&& f) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r0 = (wv >> 1) * 32, c0 = (wv & 1) * 32;
    const int li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) f(r0 + 16 * s + lk + 4 * g, c0 + 16 * t + li, acc[s][t][g]);
}

// tile row span of the rows of A (masked rows excluded): w = max over rows of (last − first tile)
__global__ __launch_bounds__(BLOCK) void k_band_width(int64_t m, const int64_t* __restrict__ rp,
                                                      const int32_t* __restrict__ ci, const int32_t* __restrict__ pinv,
                                                      const double* __restrict__ rs, int* __restrict__ wmax) {
    int local = 0;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += (int64_t)gridDim.x * BLOCK) {
        if (rs[i] == 0.0) continue;
        int lo = INT_MAX, hi = -1;
        for (int64_t f = rp[i]; f < rp[i + 1]; ++f) {
            const int k = pinv[ci[f]];
            if (k < 0) continue;   // a column outside the window (lsq_cov_band_window)
            lo = min(lo, k >> 6);
            hi = max(hi, k >> 6);
        }
        if (hi >= 0) local = max(local, hi - lo);
    }
    for (int o = 32; o > 0; o >>= 1) local = max(local, __shfl_xor(local, o));
    if ((threadIdx.x & 63) == 0 && local > 0) atomicMax(wmax, local);
}

// N = AᵀA in the new order, upper band: one thread owns row j of N (new column j = old perm[j]),
// contributions in the order of dense.hip's k_normal_rows (so every entry is the same sum)
__global__ __launch_bounds__(BLOCK) void k_band_normal(int64_t n, int64_t npad, BandDev b,
                                                       const int32_t* __restrict__ perm,
                                                       const int32_t* __restrict__ pinv,
                                                       const int64_t* __restrict__ trp, const int32_t* __restrict__ tci,
                                                       const double* __restrict__ tval, const int64_t* __restrict__ rp,
                                                       const int32_t* __restrict__ ci, const double* __restrict__ val,
                                                       const double* __restrict__ rs) {
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < npad; j += (int64_t)gridDim.x * BLOCK) {
        const int64_t I = j >> 6;
        const int rj = (int)(j & 63);
        if (j >= n) {
            btile(b.R, b.w, I, I)[rj * TB + rj] = 1.0;
            continue;
        }
        const int32_t jo = perm[j];
        for (int64_t e = trp[jo]; e < trp[jo + 1]; ++e) {
            const int32_t i = tci[e];
            const double a = tval[e] * rs[i];
            if (a == 0.0) continue;
            for (int64_t f = rp[i]; f < rp[i + 1]; ++f) {
                const int64_t k = pinv[ci[f]];
                if (k < j) continue;
                btile(b.R, b.w, I, k >> 6)[rj * TB + (k & 63)] += a * (val[f] * rs[i]);
            }
        }
    }
}

// symmetric diagonal scaling Ñ = S N S, S = diag(N)^(-1/2) (z0 and dz columns differ in scale by
// orders of magnitude; the factor of Ñ is better balanced)
__global__ __launch_bounds__(BLOCK) void k_band_dscale(BandDev b, int64_t npad, double* __restrict__ sc) {
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < npad; j += (int64_t)gridDim.x * BLOCK) {
        const int r = (int)(j & 63);
        const double d = btile(b.R, b.w, j >> 6, j >> 6)[r * TB + r];
        sc[j] = d > 0.0 ? 1.0 / sqrt(d) : 1.0;
    }
}

__global__ __launch_bounds__(BLOCK) void k_band_apply_scale(BandDev b, const double* __restrict__ sc) {
    const int64_t ntile = b.T * (b.w + 1);
    for (int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x; e < ntile * TT; e += (int64_t)gridDim.x * BLOCK) {
        const int64_t tix = e / TT;
        const int64_t I = tix / (b.w + 1), J = I + tix % (b.w + 1);
        if (J >= b.T) continue;
        const int idx = (int)(e - tix * TT);
        b.R[e] *= sc[I * TB + (idx >> 6)] * sc[J * TB + (idx & 63)];
    }
}

// broadcast lane l's double (two readlanes into scalar registers)
__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)u, l), hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// POTRF of tile (K, K), blocked by 16: per 16-column block, the 16×16 diagonal Cholesky by one
// wave (columns in registers, rows broadcast with readlane), the 16-row panel by substitution (a
// thread per trailing column), the trailing triangle's rank-16 update by all 256 threads — 12
// barriers.  (Unblocked: one wave with readlane, 68 µs per tile; 256 threads with a barrier per
// elimination step, 128 µs.)  The lower triangle is zeroed.
__device__ __forceinline__ void band_potrf_body(const BandDev& b, int64_t K, int* err) {
    __shared__ double A[TB * LDP];
    __shared__ double rinv[TB];
    __shared__ int bad;
    double* Rt = btile(b.R, b.w, K, K);
    for (int idx = threadIdx.x; idx < TT; idx += BLOCK) {
        const int r = idx >> 6, c = idx & 63;
        A[r * LDP + c] = c >= r ? Rt[idx] : 0.0;
    }
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int o = 0; o < TB; o += 16) {
        if (wv == 0) {   // 16×16 diagonal block: lane k < 16 holds its column o + k
            double a[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) a[i] = (lane < 16 && i <= lane) ? A[(o + i) * LDP + o + lane] : 0.0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const double d = readlane_d(a[j], j);
                double r = 1.0;
                if (d > 0.0) r = sqrt(d);
                else if (lane == 0) bad = 1;
                a[j] = lane == j ? r : (lane > j ? a[j] / r : 0.0);
#pragma unroll
                for (int i = j + 1; i < 16; ++i) {
                    const double rji = readlane_d(a[j], i);
                    if (lane >= i) a[i] -= rji * a[j];
                }
            }
            if (lane < 16) {
#pragma unroll
                for (int i = 0; i < 16; ++i) A[(o + i) * LDP + o + lane] = i <= lane ? a[i] : 0.0;
            }
        }
        __syncthreads();
        if (threadIdx.x < 16) rinv[o + threadIdx.x] = 1.0 / A[(o + threadIdx.x) * LDP + o + threadIdx.x];
        const int c0 = o + 16, nc = TB - c0;
        if (nc == 0) break;
        __syncthreads();
        if (threadIdx.x < nc) {   // panel: rows o..o+15 of column c, R_bbᵀ X = A by substitution
            const int c = c0 + threadIdx.x;
            double x[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = A[(o + i) * LDP + c];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                x[i] *= rinv[o + i];
#pragma unroll
                for (int q = i + 1; q < 16; ++q) x[q] -= A[(o + i) * LDP + o + q] * x[i];
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) A[(o + i) * LDP + c] = x[i];
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < nc * nc; idx += BLOCK) {   // trailing: A_ic −= Σ_p P_pi P_pc
            const int i = c0 + idx / nc, c = c0 + idx % nc;
            if (c < i) continue;
            double sum = 0.0;
#pragma unroll
            for (int q = 0; q < 16; ++q) sum += A[(o + q) * LDP + i] * A[(o + q) * LDP + c];
            A[i * LDP + c] -= sum;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && bad) atomicExch(err, 1);
    for (int idx = threadIdx.x; idx < TT; idx += BLOCK) {
        const int r = idx >> 6, c = idx & 63;
        Rt[idx] = c >= r ? A[r * LDP + c] : 0.0;
    }
}
__global__ __launch_bounds__(BLOCK) void k_band_potrf(BandDev b, int64_t K, int* err) { band_potrf_body(b, K, err); }
// a batch of bands (compute_E windows): band blockIdx.y, its error flag errs[2·y]
__global__ __launch_bounds__(BLOCK) void k_band_potrf_b(const BandDev* __restrict__ bs, int64_t K, int* errs) {
    const BandDev b = bs[blockIdx.y];
    if (K < b.T) band_potrf_body(b, K, errs + 2 * blockIdx.y);
}

// D_K = R_KK⁻¹ for every tile row at once (one wave per tile, lane k: column k by back
// substitution, R's rows broadcast with readlane)
__device__ __forceinline__ void band_dinv_body(const BandDev& b, int64_t K) {
    const int k = threadIdx.x;
    const double* Rt = btile(b.R, b.w, K, K);
    double a[TB];
#pragma unroll
    for (int i = 0; i < TB; ++i) a[i] = Rt[i * TB + k];   // column k of R (zero below the diagonal)
    double x[TB];
#pragma unroll
    for (int i = TB - 1; i >= 0; --i) {
        double s = i == k ? 1.0 : 0.0;
#pragma unroll
        for (int j = i + 1; j < TB; ++j) s -= readlane_d(a[i], j) * x[j];
        x[i] = s / readlane_d(a[i], i);
    }
    double* Dk = b.D + K * TT;
#pragma unroll
    for (int i = 0; i < TB; ++i) Dk[i * TB + k] = x[i];
}
__global__ __launch_bounds__(TB) void k_band_dinv(BandDev b) { band_dinv_body(b, blockIdx.x); }
__global__ __launch_bounds__(TB) void k_band_dinv_b(const BandDev* __restrict__ bs) {
    const BandDev b = bs[blockIdx.y];
    if ((int64_t)blockIdx.x < b.T) band_dinv_body(b, blockIdx.x);
}

// R_KJ = R_KK⁻ᵀ N_KJ for J = K+1..K+m (one workgroup per tile), blocked by 16 rows: the 16 rows
// of a block by substitution (a thread per column), then the rows below updated with them by all
// 256 threads — 8 barriers.  Multiplying by the explicit D_Kᵀ instead would lose ~cond(R_KK)·ε
// per tile row.
__device__ __forceinline__ void band_trsm_body(const BandDev& b, int64_t K, int bx) {
    __shared__ double R[TB * LDP];
    __shared__ double X[TB * LDP];
    __shared__ double rinv[TB];
    const double* Rkk = btile(b.R, b.w, K, K);
    double* Nt = btile(b.R, b.w, K, K + 1 + bx);
    for (int idx = threadIdx.x; idx < TT; idx += BLOCK) {
        const int r = idx >> 6, c = idx & 63;
        R[r * LDP + c] = Rkk[idx];
        X[r * LDP + c] = Nt[idx];
    }
    __syncthreads();
    if (threadIdx.x < TB) rinv[threadIdx.x] = 1.0 / R[threadIdx.x * LDP + threadIdx.x];
    __syncthreads();
    for (int o = 0; o < TB; o += 16) {
        if (threadIdx.x < TB) {
            const int c = threadIdx.x;
            double x[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = X[(o + i) * LDP + c];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                x[i] *= rinv[o + i];
#pragma unroll
                for (int q = i + 1; q < 16; ++q) x[q] -= R[(o + i) * LDP + o + q] * x[i];
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) X[(o + i) * LDP + c] = x[i];
        }
        __syncthreads();
        const int r0 = o + 16, nr = TB - r0;
        for (int idx = threadIdx.x; idx < nr * TB; idx += BLOCK) {   // X_pc −= Σ_i R_ip X_ic
            const int pr = r0 + (idx >> 6), c = idx & 63;
            double sum = 0.0;
#pragma unroll
            for (int i = 0; i < 16; ++i) sum += R[(o + i) * LDP + pr] * X[(o + i) * LDP + c];
            X[pr * LDP + c] -= sum;
        }
        __syncthreads();
    }
    for (int idx = threadIdx.x; idx < TT; idx += BLOCK) Nt[idx] = X[(idx >> 6) * LDP + (idx & 63)];
}
__global__ __launch_bounds__(BLOCK) void k_band_trsm(BandDev b, int64_t K) { band_trsm_body(b, K, blockIdx.x); }
__global__ __launch_bounds__(BLOCK) void k_band_trsm_b(const BandDev* __restrict__ bs, int64_t K) {
    const BandDev b = bs[blockIdx.y];
    if (K < b.T && (int64_t)blockIdx.x < std::min<int64_t>(b.w, b.T - 1 - K)) band_trsm_body(b, K, blockIdx.x);
}

// N_{K+a, K+c} −= R_{K,K+a}ᵀ R_{K,K+c}, 1 ≤ a ≤ c ≤ m, one workgroup per pair.  ROW: only the
// next tile row (a = 1, c = 1 + blockIdx.x) — the look-ahead the next POTRF/TRSM wait for;
// otherwise the rest (2 ≤ a ≤ c ≤ m, (m−1)m/2 workgroups), which runs beside them on a second
// stream.  (A square m² grid with the lower pairs idle cost ~2× in dispatch at w = 65.)
template <bool ROW>
__device__ __forceinline__ void band_syrk_body(const BandDev& b, int64_t K, int m, int bx) {
    int a = 1, c = 1 + bx;
    if (!ROW) {
        const int p = bx;
        int c0 = (int)((sqrt(8.0 * p + 1.0) - 1.0) * 0.5);
        while ((c0 + 1) * (c0 + 2) / 2 <= p) ++c0;
        while (c0 * (c0 + 1) / 2 > p) --c0;
        a = p - c0 * (c0 + 1) / 2 + 2;
        c = c0 + 2;
    }
    if (c > m) return;   // a batch's band with fewer trailing tiles than the launch's widest
    __shared__ double A[TB * LDP];
    __shared__ double B[TB * LDP];
    TilePair tp;   // both tiles' loads in flight together; A used transposed in place (no LDS transpose)
    tp.load(btile(b.R, b.w, K, K + a), btile(b.R, b.w, K, K + c));
    tp.store(A, B);
    __syncthreads();
    d4 acc[2][2];
    acc_zero(acc);
    mma_tile<true>(A, B, acc);
    double* Ct = btile(b.R, b.w, K + a, K + c);
    acc_each(acc, [&](int r, int cc, double v) { Ct[r * TB + cc] -= v; });
}
template <bool ROW>
__global__ __launch_bounds__(BLOCK) void k_band_syrk(BandDev b, int64_t K, int m) { band_syrk_body<ROW>(b, K, m, blockIdx.x); }
template <bool ROW>
__global__ __launch_bounds__(BLOCK) void k_band_syrk_b(const BandDev* __restrict__ bs, int64_t K) {
    const BandDev b = bs[blockIdx.y];
    if (K < b.T) band_syrk_body<ROW>(b, K, (int)std::min<int64_t>(b.w, b.T - 1 - K), blockIdx.x);
}

// y = R⁻ᵀ o for the 64 right-hand sides of one workgroup, tile row by tile row from the first
// non-zero row K0: Y_K = D_Kᵀ (O_K − Σ_{I=max(K0,K−w)}^{K−1} R_IKᵀ Y_I); out = ‖y‖² per right-hand
// side.  Only the last w+1 tiles of y are live: a ring per workgroup (the __threadfence closing
// each step also invalidates this CU's L1, so a rewritten slot is read fresh).
// IDENT: o = e_{64J..64J+63}, J = j0 + blockIdx.x, or J = sp[blockIdx.x] when sp is given (the
// tiles of a window's interior), out at tile J (the diagonal of N⁻¹).  Otherwise op rows: the
// workgroup's segments [sp[rt], sp[rt+1]) each hold one tile row segK[s] and the entries
// [segE[s], segE[s+1]) as (row-in-tile << 6 | rhs) in el and the value in ev (× s_j here).
template <bool IDENT>
__global__ __launch_bounds__(BLOCK) void k_band_sweep(BandDev b, int64_t j0, const int64_t* __restrict__ sp,
                                                      const int64_t* __restrict__ segK,
                                                      const int64_t* __restrict__ segE, const int32_t* __restrict__ el,
                                                      const double* __restrict__ ev, const double* __restrict__ sc,
                                                      double* __restrict__ ring, double* __restrict__ out) {
    __shared__ double A[TB * LDP];
    __shared__ double B[TB * LDP];
    __shared__ double red[4][4][2][16];
    const int64_t rt = blockIdx.x;
    const int64_t W1 = b.w + 1;
    double* Rg = ring + rt * W1 * TT;
    int64_t s = 0, s1 = 0, K0 = 0;
    if (IDENT) {
        K0 = sp ? sp[rt] : j0 + rt;
    } else {
        s = sp[rt];
        s1 = sp[rt + 1];
        K0 = segK[s];
    }
    double ss[2] = {0.0, 0.0};
    TilePair tp;
    for (int64_t K = K0; K < b.T; ++K) {
        d4 acc[2][2];
        acc_zero(acc);
        const int64_t I0 = max<int64_t>(K0, K - b.w);
        if (I0 < K) tp.load(btile(b.R, b.w, I0, K), Rg + (I0 % W1) * TT);
        for (int64_t I = I0; I < K; ++I) {
            __syncthreads();
            tp.store(A, B);
            __syncthreads();
            if (I + 1 < K) tp.load(btile(b.R, b.w, I + 1, K), Rg + ((I + 1) % W1) * TT);
            mma_tile<true>(A, B, acc);
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < TT; idx += BLOCK) {
            const int r = idx >> 6, c = idx & 63;
            B[r * LDP + c] = (IDENT && K == K0 && r == c) ? 1.0 : 0.0;
            A[r * LDP + c] = b.D[K * TT + idx];
        }
        if (!IDENT && s < s1 && segK[s] == K) {
            __syncthreads();
            for (int64_t e = segE[s] + threadIdx.x; e < segE[s + 1]; e += BLOCK) {
                const int p = el[e];
                B[(p >> 6) * LDP + (p & 63)] = ev[e] * sc[K * TB + (p >> 6)];
            }
            ++s;
        }
        __syncthreads();
        acc_each(acc, [&](int r, int c, double v) { B[r * LDP + c] -= v; });
        __syncthreads();
        acc_zero(acc);
        mma_tile<true>(A, B, acc);   // D_Kᵀ · X
        double* Yk = Rg + (K % W1) * TT;
        acc_each(acc, [&](int r, int c, double v) {
            Yk[r * TB + c] = v;
            ss[((c & 31) >= 16) ? 1 : 0] += v * v;
        });
        __threadfence();
        // the next step's first ring load (before its loop's barrier) may read this very slot
        // (step K0 + 1 reads Y_K0): every thread's stores must have landed
        __syncthreads();
    }
    // column sums: thread (wave wv, lane) holds columns c0 + 16t + (lane&15) over rows lk + 4g (+16s)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    red[wv][lane >> 4][0][lane & 15] = ss[0];
    red[wv][lane >> 4][1][lane & 15] = ss[1];
    __syncthreads();
    if (threadIdx.x < TB) {
        const int c = threadIdx.x;
        const int half = c >> 5, t = (c & 31) >> 4, li = c & 15;
        double sum = 0.0;
        for (int wr = 0; wr < 2; ++wr)
            for (int lk = 0; lk < 4; ++lk) sum += red[wr * 2 + half][lk][t][li];
        out[(IDENT ? K0 : rt) * TB + c] = sum;
    }
}

// The identity sweeps (the diagonal of N⁻¹): NC of a tile's 64 right-hand sides per workgroup,
// TB / NC workgroups per tile.  Wave v takes output rows 16v … 16v + 15 and all NC columns, with
// two MFMA chains per 16-column tile (k parity).  Measured at 256²×12 with one lane (t256,
// `gpurun_out/r5s`; the k_band_sweep layout before it took 10.6–10.8 s):
//   NC = 64 (default)   10.3 s
//   NC = 32             11.3 s
//   NC = 16             14.9 s
// Each chunk reads the R tiles again, and the sweeps are bound by the bytes they move.  PMC
// (r5q2): every tile comes from beyond L2, 2.3 TB/s.  Neither a second pair of tiles in flight
// nor two waves per SIMD moved the time (r5r, r5r2).
template <int NC>
__global__ __launch_bounds__(BLOCK) void k_band_sweep_id(BandDev b, int64_t j0, const int64_t* __restrict__ sp,
                                                         double* __restrict__ ring, double* __restrict__ out) {
    constexpr int NCH = TB / NC, LDB = NC + 1, NT = NC / 16;
    constexpr int NA = (int)(TT / 2 / BLOCK), NBV = TB * NC / 2 / BLOCK;
    __shared__ double A[TB * LDP];
    __shared__ double B[TB * LDB];
    __shared__ double red[4][4][NC];
    const int64_t rt = blockIdx.x / NCH;
    const int ch = (int)(blockIdx.x % NCH);
    const int64_t K0 = sp ? sp[rt] : j0 + rt;
    const int64_t W1 = b.w + 1, YT = (int64_t)TB * NC;   // a ring slot: 64 rows × NC columns
    double* Rg = ring + (int64_t)blockIdx.x * W1 * YT;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, li = lane & 15, lk = lane >> 4;
    const int r0 = wv * 16;
    double2 ra[NA], rb[NBV];
    auto load = [&](int64_t I, int64_t K) {
        const double2* a2 = reinterpret_cast<const double2*>(btile(b.R, b.w, I, K));
        const double2* b2 = reinterpret_cast<const double2*>(Rg + (I % W1) * YT);
#pragma unroll
        for (int i = 0; i < NA; ++i) ra[i] = a2[threadIdx.x + BLOCK * i];
#pragma unroll
        for (int i = 0; i < NBV; ++i) rb[i] = b2[threadIdx.x + BLOCK * i];
    };
    auto store = [&]() {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int idx = 2 * (threadIdx.x + BLOCK * i), r = idx >> 6, c = idx & 63;
            A[r * LDP + c] = ra[i].x;
            A[r * LDP + c + 1] = ra[i].y;
        }
#pragma unroll
        for (int i = 0; i < NBV; ++i) {
            const int idx = 2 * (threadIdx.x + BLOCK * i), r = idx / NC, c = idx % NC;
            B[r * LDB + c] = rb[i].x;
            B[r * LDB + c + 1] = rb[i].y;
        }
    };
    // acc[t][par] += Aᵀ B over the wave's rows, 16-column tile t, k parity par
    auto mma = [&](d4 (&acc)[NT][2]) {
#pragma unroll 4
        for (int k0 = 0; k0 < TB; k0 += 4) {
            const int k = k0 + lk, par = (k0 >> 2) & 1;
            const double a = A[k * LDP + r0 + li];
#pragma unroll
            for (int t = 0; t < NT; ++t)
                acc[t][par] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, B[k * LDB + 16 * t + li], acc[t][par], 0, 0, 0);
        }
    };
    auto zero = [&](d4 (&acc)[NT][2]) {
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t][0] = acc[t][1] = d4{0.0, 0.0, 0.0, 0.0};
    };
    double ss[NT] = {};
    for (int64_t K = K0; K < b.T; ++K) {
        d4 acc[NT][2];
        zero(acc);
        const int64_t I0 = max<int64_t>(K0, K - b.w);
        if (I0 < K) load(I0, K);
        for (int64_t I = I0; I < K; ++I) {
            __syncthreads();
            store();
            __syncthreads();
            if (I + 1 < K) load(I + 1, K);
            mma(acc);
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < TT; idx += BLOCK) A[(idx >> 6) * LDP + (idx & 63)] = b.D[K * TT + idx];
        for (int idx = threadIdx.x; idx < TB * NC; idx += BLOCK) {
            const int r = idx / NC, c = idx % NC;
            B[r * LDB + c] = (K == K0 && r == ch * NC + c) ? 1.0 : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) B[(r0 + lk + 4 * g) * LDB + 16 * t + li] -= acc[t][0][g] + acc[t][1][g];
        __syncthreads();
        zero(acc);
        mma(acc);   // D_Kᵀ · X
        double* Yk = Rg + (K % W1) * YT;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const double v = acc[t][0][g] + acc[t][1][g];
                Yk[(r0 + lk + 4 * g) * NC + 16 * t + li] = v;
                ss[t] += v * v;
            }
        __threadfence();
        // the next step's first ring load (before its loop's barrier) may read this very slot
        // (step K0 + 1 reads Y_K0): every thread's stores must have landed
        __syncthreads();
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) red[wv][lk][16 * t + li] = ss[t];
    __syncthreads();
    if (threadIdx.x < NC) {
        const int c = threadIdx.x;
        double sum = 0.0;
        for (int w = 0; w < 4; ++w)
            for (int l = 0; l < 4; ++l) sum += red[w][l][c];
        out[K0 * TB + ch * NC + c] = sum;
    }
}

// E[perm[j]] = sqrt(ss_j)·s_j from the identity sweeps (perm null: E[j], window order)
__global__ __launch_bounds__(BLOCK) void k_band_diag_sweep(int64_t n, const int32_t* __restrict__ perm,
                                                           const double* __restrict__ ssq,
                                                           const double* __restrict__ sc, double* __restrict__ E) {
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK)
        E[perm ? perm[j] : j] = sqrt(ssq[j]) * sc[j];
}

// ---- precond 5: LSQR on A·M, M = P·S·R̃⁻¹ (lsqr.hip) ------------------------------------------
// A triangular solve is a chain of T dependent tile steps.  NW workgroups (one per CU, all
// resident: NW ≤ 64 on a 256-CU device) split each step's w band tiles, publish their partial
// 64-vectors, meet at a grid barrier, and every workgroup then finishes the step redundantly
// (sum of the partials in a fixed order, the 64×64 diagonal-block product), keeping the last w+1
// solved tiles in its own LDS ring.  One barrier per step; the partials are double-buffered by
// step parity (a workgroup can be at most one barrier ahead).  A single workgroup streamed the
// band at ~45 GB/s (3 s per solve at 2048²).

struct GridBar {
    unsigned int count, gen;
    int err, pad;
};

// all NW workgroups of the launch meet; false when a barrier timed out (then every workgroup
// leaves its loop: a bounded spin, so a launch that is not co-resident fails instead of hanging)
__device__ __forceinline__ bool grid_barrier(GridBar* g, unsigned int nwg, unsigned int& gen) {
    __shared__ int ok;
    __threadfence();   // every thread's partial-sum stores, before the workgroup arrives
    __syncthreads();
    if (threadIdx.x == 0) {
        ok = 1;
        __threadfence();
        const unsigned int arrived = atomicAdd(&g->count, 1u) + 1u;
        if (arrived == nwg) {
            atomicExch(&g->count, 0u);
            __threadfence();
            atomicAdd(&g->gen, 1u);
        } else {
            long spins = 0;
            while (__hip_atomic_load(&g->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen) {
                if (++spins > (1L << 24) || __hip_atomic_load(&g->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    atomicExch(&g->err, 1);
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        ++gen;
    }
    __syncthreads();
    return ok != 0;
}

// out = M·v·scale: x̃ = R̃⁻¹ v by back substitution, x̃_K = D_K (v_K − Σ_{J=K+1}^{K+w} R̃_KJ x̃_J),
// out[perm[j]] = sc_j x̃_j.  scale_mode 1: v / α (and nothing once the solve stopped), 2: v.
// Workgroup p takes the tiles J − K − 1 ≡ p (mod NW); thread (r = t/4, q = t%4) a 16-wide
// segment of row r of each.  The next step's first tile and D_K segment are loaded before the
// barrier (they do not depend on x), so their latency hides behind it.
__global__ __launch_bounds__(BLOCK) void k_band_bsub(const double* __restrict__ R, const double* __restrict__ D,
                                                     int64_t T, int w, int64_t n, const double* __restrict__ v,
                                                     const LsqState* __restrict__ st, int scale_mode,
                                                     const double* __restrict__ sc, const int32_t* __restrict__ perm,
                                                     double* __restrict__ out, double* __restrict__ part,
                                                     GridBar* __restrict__ bar) {
    if (st && st->stop && scale_mode != 2) return;
    extern __shared__ double ring[];   // (w+1) × 64
    __shared__ double Y[TB];
    const unsigned int NW = gridDim.x, p = blockIdx.x;
    unsigned int gen = 0;
    const double scale = scale_mode == 1 ? st->inv_alpha : 1.0;
    const int t = threadIdx.x, r = t >> 2, q = t & 3;
    double2 rn[8];   // row segment of the next step's first tile (zeros when there is none)
    double dn[16];   // row segment of the next step's D
    auto fetch = [&](int64_t K) {
        const int64_t J = K + 1 + p;
        const bool has = K >= 0 && J <= min<int64_t>(K + w, T - 1);
        const double2* Rt = reinterpret_cast<const double2*>(R + ((K * (w + 1)) + (J - K)) * TT + r * TB + q * 16);
#pragma unroll
        for (int c = 0; c < 8; ++c) rn[c] = has ? Rt[c] : make_double2(0.0, 0.0);
        const double* Dr = D + (K >= 0 ? K : 0) * TT + r * TB + q * 16;
#pragma unroll
        for (int c = 0; c < 16; ++c) dn[c] = K >= 0 ? Dr[c] : 0.0;
    };
    fetch(T - 1);
    for (int64_t K = T - 1; K >= 0; --K) {
        double acc = 0.0;
        const int64_t J1 = min<int64_t>(K + w, T - 1);
        if (K + 1 + p <= J1) {   // (the ring slot of a tile that does not exist may hold garbage)
            const double* xs = ring + ((K + 1 + p) % (w + 1)) * TB + q * 16;
#pragma unroll
            for (int c = 0; c < 8; ++c) acc += rn[c].x * xs[2 * c] + rn[c].y * xs[2 * c + 1];
        }
        for (int64_t J = K + 1 + p + NW; J <= J1; J += NW) {   // further tiles when NW < w
            const double2* Rt = reinterpret_cast<const double2*>(R + ((K * (w + 1)) + (J - K)) * TT + r * TB + q * 16);
            const double* xs = ring + (J % (w + 1)) * TB + q * 16;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const double2 a = Rt[c];
                acc += a.x * xs[2 * c] + a.y * xs[2 * c + 1];
            }
        }
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        double* pb = part + (K & 1) * NW * TB;
        if (q == 0) pb[p * TB + r] = acc;
        double dk[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) dk[c] = dn[c];
        fetch(K - 1);
        if (NW > 1 && !grid_barrier(bar, NW, gen)) return;
        const int64_t j = K * TB + r;
        if (q == 0) {
            double sum = 0.0;
            for (unsigned int pp = 0; pp < NW; ++pp) sum += pb[pp * TB + r];
            Y[r] = (j < n ? v[j] * scale : 0.0) - sum;
        }
        __syncthreads();
        double x = 0.0;   // x̃_K = D_K Y (D upper)
#pragma unroll
        for (int c = 0; c < 16; ++c) x += dk[c] * Y[q * 16 + c];
        x += __shfl_xor(x, 1);
        x += __shfl_xor(x, 2);
        if (q == 0) {
            ring[(K % (w + 1)) * TB + r] = x;
            if (p == 0 && j < n) out[perm[j]] = sc[j] * x;
        }
        __syncthreads();
    }
}

// vout = R̃⁻ᵀ (S Pᵀ t) with LSQR's epilogue (as dense.hip's k_gemvT_upper mode 1):
// ỹ_K = D_Kᵀ (t̃_K − Σ_{I=K−w}^{K−1} R̃_IKᵀ ỹ_I), vout_j = ỹ_j/β − β vin_j/α (vin_j when β = 0),
// part[0] = Σ vout².  Workgroup p takes the tiles K − 1 − I ≡ p (mod NW); thread (c = t%64,
// q = t/64) rows q·16 .. q·16+15 of column c of each; the next step's first tile and D column
// segment are loaded before the barrier.
__global__ __launch_bounds__(BLOCK) void k_band_fsub(const double* __restrict__ R, const double* __restrict__ D,
                                                     int64_t T, int w, int64_t n, const double* __restrict__ tin,
                                                     const LsqState* __restrict__ st, const double* __restrict__ vin,
                                                     double* __restrict__ vout, const double* __restrict__ sc,
                                                     const int32_t* __restrict__ perm, double* __restrict__ part,
                                                     double* __restrict__ pv, GridBar* __restrict__ bar) {
    if (st && st->stop) return;
    extern __shared__ double ring[];   // (w+1) × 64
    __shared__ double Z[TB];
    __shared__ double P4[4][TB];
    __shared__ double red[4];
    const unsigned int NW = gridDim.x, p = blockIdx.x;
    unsigned int gen = 0;
    const int t = threadIdx.x, c = t & 63, q = t >> 6;
    double rn[16], dn[16];
    auto fetch = [&](int64_t K) {
        const int64_t I = K - 1 - p;
        const bool has = K < T && I >= max<int64_t>(0, K - w);
        const double* Rt = R + ((I * (w + 1)) + (K - I)) * TT + (q * 16) * TB + c;
#pragma unroll
        for (int r = 0; r < 16; ++r) rn[r] = has ? Rt[r * TB] : 0.0;
        const double* Dc = D + (K < T ? K : 0) * TT + (q * 16) * TB + c;
#pragma unroll
        for (int r = 0; r < 16; ++r) dn[r] = K < T ? Dc[r * TB] : 0.0;
    };
    double sv = 0.0;
    fetch(0);
    for (int64_t K = 0; K < T; ++K) {
        double acc = 0.0;
        {
            const int64_t I = K - 1 - p;
            if (I >= max<int64_t>(0, K - w)) {
                const double* ys = ring + (I % (w + 1)) * TB + q * 16;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc += rn[r] * ys[r];
            }
        }
        for (int64_t I = K - 1 - p - NW; I >= max<int64_t>(0, K - w); I -= NW) {
            const double* Rt = R + ((I * (w + 1)) + (K - I)) * TT + (q * 16) * TB + c;
            const double* ys = ring + (I % (w + 1)) * TB + q * 16;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc += Rt[r * TB] * ys[r];
        }
        double dk[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) dk[r] = dn[r];
        fetch(K + 1);
        P4[q][c] = acc;
        __syncthreads();
        double* pb = part + (K & 1) * NW * TB;
        if (q == 0) pb[p * TB + c] = (P4[0][c] + P4[1][c]) + (P4[2][c] + P4[3][c]);
        if (NW > 1 && !grid_barrier(bar, NW, gen)) return;
        const int64_t j = K * TB + c;
        if (q == 0) {
            double sum = 0.0;
            for (unsigned int pp = 0; pp < NW; ++pp) sum += pb[pp * TB + c];
            Z[c] = (j < n ? tin[perm[j]] * sc[j] : 0.0) - sum;
        }
        __syncthreads();
        double y = 0.0;   // (D_Kᵀ Z)_c = Σ_r D[r][c] Z[r]
#pragma unroll
        for (int r = 0; r < 16; ++r) y += dk[r] * Z[q * 16 + r];
        P4[q][c] = y;
        __syncthreads();
        if (q == 0) {
            const double yc = (P4[0][c] + P4[1][c]) + (P4[2][c] + P4[3][c]);
            ring[(K % (w + 1)) * TB + c] = yc;
            if (p == 0 && j < n) {
                const double o = st->skip_v ? vin[j] : yc * st->inv_beta - st->beta * (vin[j] * st->inv_alpha);
                vout[j] = o;
                sv += o * o;
            }
        }
        __syncthreads();
    }
    const double s = block_sum(sv, red);
    if (p == 0 && threadIdx.x == 0) pv[0] = s;
}

// warm start y0 = M⁻¹ x0 = R̃ S⁻¹ Pᵀ x0 (one thread per row of R̃)
__global__ __launch_bounds__(BLOCK) void k_band_warm(const double* __restrict__ R, int64_t T, int w, int64_t n,
                                                     const double* __restrict__ x0, const double* __restrict__ sc,
                                                     const int32_t* __restrict__ perm, double* __restrict__ y0) {
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK) {
        const int64_t I = j >> 6;
        const int rj = (int)(j & 63);
        double s = 0.0;
        for (int64_t J = I; J <= min<int64_t>(I + w, T - 1); ++J) {
            const double* row = R + ((I * (w + 1)) + (J - I)) * TT + rj * TB;
            for (int c = (J == I ? rj : 0); c < TB; ++c) {
                const int64_t k = J * TB + c;
                if (k < n) s += row[c] * (x0[perm[k]] / sc[k]);
            }
        }
        y0[j] = s;
    }
}

}  // namespace

namespace {

// op rows (new column order) as sweep right-hand sides: 64 rows per workgroup, entries grouped by
// tile row (segments), each workgroup starting at its first non-zero tile row
struct SweepOps {
    std::vector<int64_t> sp{0}, segK, segE{0};
    std::vector<int32_t> el;
    std::vector<double> ev;
    int64_t gemms = 0;
};

// pinv: compact column -> position (null: ci already holds positions)
SweepOps sweep_ops(const std::vector<int64_t>& rows, const int64_t* rp, const int32_t* ci, const double* v,
                   const int32_t* pinv, int64_t T, int w) {
    SweepOps o;
    struct Ent { int64_t K; int32_t p; double v; };
    for (size_t r0 = 0; r0 < rows.size(); r0 += TB) {
        std::vector<Ent> ents;
        for (size_t q = r0; q < std::min(rows.size(), r0 + TB); ++q)
            for (int64_t e = rp[rows[q]]; e < rp[rows[q] + 1]; ++e) {
                const int64_t j = pinv ? pinv[ci[e]] : ci[e];
                ents.push_back({j >> 6, (int32_t)(((j & 63) << 6) | (int64_t)(q - r0)), v[e]});
            }
        std::stable_sort(ents.begin(), ents.end(), [](const Ent& a, const Ent& b) { return a.K < b.K; });
        if (ents.empty()) ents.push_back({T - 1, 0, 0.0});   // an all-zero row block: one trivial step
        for (size_t e = 0; e < ents.size(); ++e) {
            if (e == 0 || ents[e].K != ents[e - 1].K) {
                if (e) o.segE.push_back((int64_t)o.el.size());
                o.segK.push_back(ents[e].K);
            }
            o.el.push_back(ents[e].p);
            o.ev.push_back(ents[e].v);
        }
        o.segE.push_back((int64_t)o.el.size());
        o.sp.push_back((int64_t)o.segK.size());
        o.gemms += (T - ents.front().K) * (int64_t)(w + 1);
    }
    return o;
}

// The tile steps of the band Cholesky, asynchronous on st (+ side): look-ahead — step K's POTRF,
// TRSM and next-row update on st; the rest of its trailing update (rows K+2..) on side, joined
// before the next-row update of K+1; then D_K = R_KK⁻¹ for every tile row.  err: non-positive pivot.
void band_factor_steps(const BandDev& b, hipStream_t st, hipStream_t side, hipEvent_t fork, hipEvent_t join, int* err) {
    const int64_t T = b.T;
    const int w = b.w;
    HIP_CHECK(hipEventRecord(join, st));
    for (int64_t K = 0; K < T; ++K) {
        hipLaunchKernelGGL(k_band_potrf, dim3(1), dim3(BLOCK), 0, st, b, K, err);
        const int m = (int)std::min<int64_t>(w, T - 1 - K);
        if (m > 0) {
            hipLaunchKernelGGL(k_band_trsm, dim3(m), dim3(BLOCK), 0, st, b, K);
            HIP_CHECK(hipStreamWaitEvent(st, join, 0));
            hipLaunchKernelGGL(k_band_syrk<true>, dim3(m), dim3(BLOCK), 0, st, b, K, m);
            if (m > 1) {
                HIP_CHECK(hipEventRecord(fork, st));
                HIP_CHECK(hipStreamWaitEvent(side, fork, 0));
                hipLaunchKernelGGL(k_band_syrk<false>, dim3((m - 1) * m / 2), dim3(BLOCK), 0, side, b, K, m);
                HIP_CHECK(hipEventRecord(join, side));
            }
        }
    }
    HIP_CHECK(hipStreamWaitEvent(st, join, 0));
    hipLaunchKernelGGL(k_band_dinv, dim3((unsigned)T), dim3(TB), 0, st, b);
    KERNEL_CHECK();
}

// The same steps for a batch of independent bands (compute_E's windows): one launch per kernel
// and step serves every band of the batch (blockIdx.y), so the chain's latency — a window's
// factorization is T dependent steps of 1–w workgroups — is paid once per batch, not per window.
// d_bs: the bands on the device, bs: the same on the host; errs: 2 ints per band ([0] pivot).
void band_factor_steps_batch(const BandDev* d_bs, const std::vector<BandDev>& bs, hipStream_t st, hipStream_t side,
                             hipEvent_t fork, hipEvent_t join, int* errs) {
    const unsigned nb = (unsigned)bs.size();
    int64_t Tmax = 0;
    for (const BandDev& b : bs) Tmax = std::max(Tmax, b.T);
    HIP_CHECK(hipEventRecord(join, st));
    for (int64_t K = 0; K < Tmax; ++K) {
        hipLaunchKernelGGL(k_band_potrf_b, dim3(1, nb), dim3(BLOCK), 0, st, d_bs, K, errs);
        int m = 0;
        for (const BandDev& b : bs)
            if (K < b.T) m = std::max<int>(m, (int)std::min<int64_t>(b.w, b.T - 1 - K));
        if (m > 0) {
            hipLaunchKernelGGL(k_band_trsm_b, dim3(m, nb), dim3(BLOCK), 0, st, d_bs, K);
            HIP_CHECK(hipStreamWaitEvent(st, join, 0));
            hipLaunchKernelGGL(k_band_syrk_b<true>, dim3(m, nb), dim3(BLOCK), 0, st, d_bs, K);
            if (m > 1) {
                HIP_CHECK(hipEventRecord(fork, st));
                HIP_CHECK(hipStreamWaitEvent(side, fork, 0));
                hipLaunchKernelGGL(k_band_syrk_b<false>, dim3((m - 1) * m / 2, nb), dim3(BLOCK), 0, side, d_bs, K);
                HIP_CHECK(hipEventRecord(join, side));
            }
        }
    }
    HIP_CHECK(hipStreamWaitEvent(st, join, 0));
    hipLaunchKernelGGL(k_band_dinv_b, dim3((unsigned)Tmax, nb), dim3(TB), 0, st, d_bs);
    KERNEL_CHECK();
}

__global__ __launch_bounds__(BLOCK) void k_band_pinv(int64_t n, const int32_t* __restrict__ perm,
                                                     int32_t* __restrict__ pinv) {
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK) pinv[perm[j]] = (int32_t)j;
}

// the identity sweeps' column chunk (k_band_sweep_id; -DBAND_NC=32/16 at build time, A/B)
#ifndef BAND_NC
#define BAND_NC 64
#endif
// launch the sweeps of `nwg` workgroups in batches whose rings fit `ring` (cap workgroups each;
// the identity sweeps: cap tiles, each TB / BAND_NC workgroups of TB / BAND_NC of a tile's ring)
template <bool IDENT>
void run_sweeps(hipStream_t st, const BandDev& b, int64_t nwg, int64_t cap, const int64_t* sp, const int64_t* segK,
                const int64_t* segE, const int32_t* el, const double* ev, const double* sc, double* ring, double* out) {
    for (int64_t g0 = 0; g0 < nwg; g0 += cap) {
        const int64_t g = std::min(cap, nwg - g0);
        if (IDENT)   // sp: the tiles to sweep (null: tiles g0 … g0 + g − 1), BAND_NC columns per workgroup
            hipLaunchKernelGGL(k_band_sweep_id<BAND_NC>, dim3((unsigned)(g * (TB / BAND_NC))), dim3(BLOCK), 0, st, b, g0,
                               sp ? sp + g0 : nullptr, ring, out);
        else
            hipLaunchKernelGGL(k_band_sweep<false>, dim3((unsigned)g), dim3(BLOCK), 0, st, b, (int64_t)0, sp + g0, segK,
                               segE, el, ev, sc, ring, out + g0 * TB);
        KERNEL_CHECK();
    }
}

}  // namespace

// AᵀA of the current weighted, masked system in the order h_perm (nullable: natural), equilibrated
// and factored inside its band into F
// nw ≥ 0: the first nw entries of h_perm are a WINDOW of the columns; the factor is that of the
// principal submatrix (AᵀA)_WW = A_WᵀA_W (every other column held fixed)
void band_factor(System& S, const int32_t* h_perm, BandFactor& F, int64_t nw) {
    ensure_full_csr(S);   // the band of AᵀA from G / GT
    hipStream_t st = S.stream;
    const int64_t ncol = S.G.n;
    const int64_t n = nw >= 0 ? nw : ncol;
    if (n <= 0) throw std::invalid_argument("band factor: empty system");
    if (n >= INT_MAX) throw std::invalid_argument("band factor: too many columns");
    if (nw >= 0 && (!h_perm || nw > ncol)) throw std::invalid_argument("band factor: bad window");
    std::vector<int32_t> pinv(ncol, -1), perm(n);
    for (int64_t j = 0; j < n; ++j) {
        const int32_t o = h_perm ? h_perm[j] : (int32_t)j;
        if (o < 0 || o >= ncol || pinv[o] >= 0) throw std::invalid_argument("band factor: the order is not a permutation of the columns");
        pinv[o] = (int32_t)j;
        perm[j] = o;
    }
    const int64_t T = (n + TB - 1) / TB, npad = T * TB;
    DBuf<int32_t> dpinv(ncol);
    F.perm.alloc(n);
    F.perm.upload(perm.data(), n, st);
    dpinv.upload(pinv.data(), ncol, st);
    DBuf<int> wmax(1);
    wmax.zero(st);
    hipLaunchKernelGGL(k_band_width, dim3(grid_for(S.G.m)), dim3(BLOCK), 0, st, S.G.m, S.G.rp.p, S.G.ci.p, dpinv.p,
                       S.rs.p, wmax.p);
    KERNEL_CHECK();
    int hw = 0;
    HIP_CHECK(hipMemcpyAsync(&hw, wmax.p, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    const int w = (int)std::min<int64_t>(hw, T - 1);
    const int64_t band_tiles = T * (int64_t)(w + 1);
    const int64_t bytes = (band_tiles + T) * TT * (int64_t)sizeof(double);
    size_t free_b = 0, total_b = 0;
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    if ((double)bytes > 0.85 * (double)free_b)
        throw Refused("band factor: a band of " + std::to_string(w) + " tiles needs " +
                                    std::to_string(bytes >> 20) + " MiB, more than the device has free");
    F.valid = false;
    F.n = n;
    F.T = T;
    F.w = w;
    graph_cache_drop(&S);   // a captured band-preconditioned LSQR batch holds the old factor's pointers
    F.R.alloc(band_tiles * TT);
    F.D.alloc(T * TT);
    F.sc.alloc(npad);
    F.R.zero(st);
    BandDev b{T, w, F.R.p, F.D.p};
    hipLaunchKernelGGL(k_band_normal, dim3(grid_for(npad)), dim3(BLOCK), 0, st, n, npad, b, F.perm.p, dpinv.p,
                       S.GT.rp.p, S.GT.ci.p, S.GT.val.p, S.G.rp.p, S.G.ci.p, S.G.val.p, S.rs.p);
    KERNEL_CHECK();
    hipLaunchKernelGGL(k_band_dscale, dim3(grid_for(npad)), dim3(BLOCK), 0, st, b, npad, F.sc.p);
    hipLaunchKernelGGL(k_band_apply_scale, dim3(grid_for(band_tiles * TT)), dim3(BLOCK), 0, st, b, F.sc.p);
    KERNEL_CHECK();
    DBuf<int> err(1);
    err.zero(st);
    if (!S.side) {
        HIP_CHECK(hipStreamCreateWithFlags(&S.side, hipStreamNonBlocking));
        HIP_CHECK(hipEventCreateWithFlags(&S.ev_fork, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&S.ev_join, hipEventDisableTiming));
    }
    band_factor_steps(b, st, S.side, S.ev_fork, S.ev_join, err.p);
    int h_err = 0;
    HIP_CHECK(hipMemcpyAsync(&h_err, err.p, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (h_err) throw std::invalid_argument("band factor: AᵀA is not positive definite (rank-deficient system)");
    F.valid = true;
}

// precond 5 needs the ring of w+1 tile vectors in LDS
constexpr int BAND_PRECOND_WMAX = 300;

void band_precond(System& S) {
    // a refactor reallocates R, D, sc and perm: captured LSQR batches hold the old pointers
    graph_cache_drop(&S);
    band_factor(S, S.band_order.empty() ? nullptr : S.band_order.data(), S.band);
    if (S.band.w > BAND_PRECOND_WMAX) {
        S.band.valid = false;
        throw Refused("precond 5: the band of AᵀA is " + std::to_string(S.band.w) +
                                    " tiles wide (at most " + std::to_string(BAND_PRECOND_WMAX) +
                                    "); set a bandwidth-reducing order (lsq_set_band_order)");
    }
    band_solve_scratch(S);   // partial sums and barrier sized here, never inside a graph capture
}

// workgroups of the multi-workgroup triangular solves: co-resident on any device, and few — the
// barrier's arrivals are atomics on one address, which serialise (LSQ_BAND_NW; at 1025²: 8
// workgroups 0.75 s of triangular solves, 16: 0.78 s, 32 or 64: 1.05 s)
int band_nw(const BandFactor& F) {
    static const int cap = [] {
        const char* e = getenv("LSQ_BAND_NW");
        return e ? std::max(1, std::min(atoi(e), 64)) : 8;
    }();
    return std::max(1, std::min(F.w, cap));
}

void band_solve_scratch(System& S) {
    BandFactor& F = S.band;
    const int nw = band_nw(F);
    if (F.part.n < 2 * nw * TB) F.part.alloc(2 * nw * TB);
    if (!F.bar.p) {
        F.bar.alloc(2);
        F.bar.zero(S.stream);
    }
}

// a multi-workgroup solve whose barrier timed out (workgroups not co-resident) leaves err set in
// the barrier (only count / gen are reset per launch): fail loudly instead of returning garbage
void band_check(System& S) {
    if (!S.band.bar.p) return;
    GridBar h{};
    HIP_CHECK(hipMemcpyAsync(&h, S.band.bar.p, sizeof(h), hipMemcpyDeviceToHost, S.stream));
    HIP_CHECK(hipStreamSynchronize(S.stream));
    if (h.err) {
        S.band.bar.zero(S.stream);
        throw std::runtime_error("precond 5: a band triangular solve's grid barrier timed out");
    }
}

void band_launch_bsub(System& S, const double* v, int scale_mode, double* out) {
    BandFactor& F = S.band;
    band_solve_scratch(S);
    const int nw = band_nw(F);
    HIP_CHECK(hipMemsetAsync(F.bar.p, 0, 2 * sizeof(unsigned int), S.stream));   // count, gen (err is sticky)
    hipLaunchKernelGGL(k_band_bsub, dim3(nw), dim3(BLOCK), sizeof(double) * TB * (F.w + 1), S.stream, F.R.p, F.D.p,
                       F.T, F.w, F.n, v, S.st.p, scale_mode, F.sc.p, F.perm.p, out, F.part.p,
                       reinterpret_cast<GridBar*>(F.bar.p));
}

void band_launch_fsub(System& S, const double* t, const double* vin, double* vout, double* part) {
    BandFactor& F = S.band;
    band_solve_scratch(S);
    const int nw = band_nw(F);
    HIP_CHECK(hipMemsetAsync(F.bar.p, 0, 2 * sizeof(unsigned int), S.stream));   // count, gen (err is sticky)
    hipLaunchKernelGGL(k_band_fsub, dim3(nw), dim3(BLOCK), sizeof(double) * TB * (F.w + 1), S.stream, F.R.p, F.D.p,
                       F.T, F.w, F.n, t, S.st.p, vin, vout, F.sc.p, F.perm.p, F.part.p, part,
                       reinterpret_cast<GridBar*>(F.bar.p));
}

void band_launch_warm(System& S, const double* x0, double* y0) {
    const BandFactor& F = S.band;
    hipLaunchKernelGGL(k_band_warm, dim3(grid_for(F.n)), dim3(BLOCK), 0, S.stream, F.R.p, F.T, F.w, F.n, x0, F.sc.p,
                       F.perm.p, y0);
}

// sparseqr.rz drop-in (lsq_band_factor): the band factor of the current weighted, masked system in
// the order h_perm, downloaded (info = n, T, w; R_out: T·(w+1) row-major 64×64 tiles, tile (I, J)
// at (I·(w+1) + J − I)·4096, upper triangle of the diagonal tiles; sc_out: S (T·64); perm_out: n).
// Null outputs: info only.
void band_factor_download(System& S, const int32_t* h_perm, int64_t* info, double* R_out, double* sc_out,
                          int32_t* perm_out) {
    refresh_scaling(S, S.cs_mode < 0 ? 0 : S.cs_mode);
    BandFactor F;
    band_factor(S, h_perm, F);
    info[0] = F.n;
    info[1] = F.T;
    info[2] = F.w;
    if (R_out) F.R.download(R_out, F.T * (int64_t)(F.w + 1) * TT, S.stream);
    if (sc_out) F.sc.download(sc_out, F.T * TB, S.stream);
    if (perm_out) F.perm.download(perm_out, F.n, S.stream);
    HIP_CHECK(hipStreamSynchronize(S.stream));
}

void band_cov(System& S, const int32_t* h_perm, int64_t nw, double* h_E, int64_t nops, const int64_t* h_rp,
              const int32_t* h_ci, const double* h_v, double* h_oe, int64_t* info, const uint8_t* inner) {
    hipStream_t st = S.stream;
    refresh_scaling(S, S.cs_mode < 0 ? 0 : S.cs_mode);
    const int64_t ncol = S.G.n;
    for (int64_t i = 0; i < nops; ++i)
        for (int64_t e = h_rp[i]; e < h_rp[i + 1]; ++e)
            if (h_ci[e] < 0 || h_ci[e] >= ncol) throw std::invalid_argument("lsq_cov_band: op column out of range");
    const auto t0 = std::chrono::steady_clock::now();
    BandFactor F;
    band_factor(S, h_perm, F, nw);
    const auto t1 = std::chrono::steady_clock::now();
    const int64_t n = F.n, T = F.T, npad = T * TB;
    const int w = F.w;
    std::vector<int32_t> pinv(ncol, -1);
    {
        std::vector<int32_t> perm(n);
        F.perm.download(perm.data(), n, st);
        HIP_CHECK(hipStreamSynchronize(st));
        for (int64_t j = 0; j < n; ++j) pinv[perm[j]] = (int32_t)j;
    }
    for (int64_t i = 0; i < nops; ++i)
        for (int64_t e = h_rp[i]; e < h_rp[i + 1]; ++e)
            if (pinv[h_ci[e]] < 0) throw std::invalid_argument("lsq_cov_band_window: an op row reaches outside the window");
    BandDev b{T, w, F.R.p, F.D.p};
    const int64_t ring_wg = (int64_t)(w + 1) * TT * (int64_t)sizeof(double);
    const int64_t bytes = (T * (int64_t)(w + 1) + T) * TT * (int64_t)sizeof(double) + npad * 16;
    size_t free_b = 0, total_b = 0;
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    const double avail = 0.9 * (double)free_b;
    if (avail < (double)ring_wg * 64)
        throw Refused("lsq_cov_band: no device memory left for the sweeps of a " + std::to_string(w) +
                                    "-tile band");
    // rings for up to `cap` concurrent workgroups (launches are batched beyond)
    const int64_t nop_wg = (nops + TB - 1) / TB;
    const int64_t cap = std::min<int64_t>({(int64_t)(0.5 * avail / ring_wg), std::max(T, nop_wg), 1 << 16});
    DBuf<double> ring(cap * (w + 1) * TT);
    // the diagonal: identity right-hand sides, tile J from row J on — every tile, or (a window's
    // interior) the tiles holding an inner position: their sweeps are the window's whole result
    std::vector<int64_t> tiles;
    if (nw >= 0 && inner) {
        for (int64_t J = 0; J < T; ++J) {
            bool any = false;
            for (int64_t j = J * TB; j < std::min<int64_t>(n, (J + 1) * TB) && !any; ++j) any = inner[j] != 0;
            if (any) tiles.push_back(J);
        }
    } else {
        tiles.resize(T);
        for (int64_t J = 0; J < T; ++J) tiles[J] = J;
    }
    const int64_t nsw = (int64_t)tiles.size();
    const int64_t nE = nw >= 0 ? n : ncol;   // a window: E in window order
    DBuf<double> ssq(npad), dE(std::max<int64_t>(nE, 1));
    DBuf<int64_t> dtiles(std::max<int64_t>(nsw, 1));
    ssq.zero(st);   // tiles not swept: E = 0
    if (nw < 0 && n < ncol) dE.zero(st);
    if (nsw > 0) {
        dtiles.upload(tiles.data(), nsw, st);
        run_sweeps<true>(st, b, nsw, cap, dtiles.p, nullptr, nullptr, nullptr, nullptr, F.sc.p, ring.p, ssq.p);
    }
    hipLaunchKernelGGL(k_band_diag_sweep, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, nw >= 0 ? nullptr : F.perm.p,
                       ssq.p, F.sc.p, dE.p);
    KERNEL_CHECK();
    dE.download(h_E, nE, st);
    HIP_CHECK(hipStreamSynchronize(st));
    if (nw >= 0 && inner)
        for (int64_t j = 0; j < n; ++j)
            if (!inner[j]) h_E[j] = 0.0;
    int64_t products = 0;
    for (int64_t J : tiles) products += (T - J) * (int64_t)std::min<int64_t>(w + 1, T - J);
    if (nops > 0) {
        std::vector<int64_t> rows(nops);
        for (int64_t i = 0; i < nops; ++i) rows[i] = i;
        SweepOps so = sweep_ops(rows, h_rp, h_ci, h_v, pinv.data(), T, w);
        products += so.gemms;
        const int64_t nwg = (int64_t)so.sp.size() - 1;
        DBuf<int64_t> dsp(nwg + 1), dsegK((int64_t)so.segK.size()), dsegE((int64_t)so.segE.size());
        DBuf<int32_t> del(std::max<int64_t>((int64_t)so.el.size(), 1));
        DBuf<double> dev(std::max<int64_t>((int64_t)so.ev.size(), 1)), dout(nwg * TB);
        dsp.upload(so.sp.data(), nwg + 1, st);
        dsegK.upload(so.segK.data(), (int64_t)so.segK.size(), st);
        dsegE.upload(so.segE.data(), (int64_t)so.segE.size(), st);
        del.upload(so.el.data(), (int64_t)so.el.size(), st);
        dev.upload(so.ev.data(), (int64_t)so.ev.size(), st);
        run_sweeps<false>(st, b, nwg, cap, dsp.p, dsegK.p, dsegE.p, del.p, dev.p, F.sc.p, ring.p, dout.p);
        std::vector<double> o(nwg * TB);
        dout.download(o.data(), nwg * TB, st);
        HIP_CHECK(hipStreamSynchronize(st));
        for (int64_t i = 0; i < nops; ++i) h_oe[i] = std::sqrt(o[i]);
    }
    HIP_CHECK(hipStreamSynchronize(st));
    if (info) {
        info[0] = w;
        info[1] = T;
        info[2] = bytes + ring.n * (int64_t)sizeof(double);
        info[3] = products;
        info[4] = std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();   // factor (host wall)
        info[5] = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t1).count();
    }
}


// ---- a window's bottom margin eliminated first (the Schur split, lsq_cov_band_windows_schur) -----
// E of a window's interior only needs the factor of the Schur complement of the margin onto the
// interior: with the columns [Mt (top margin rows), I (interior rows), Mb (bottom margin rows)] and
// Mt, Mb uncoupled, (N⁻¹)_II = S⁻¹, S = N_II − N_I,Mt N_Mt⁻¹ N_Mt,I − N_I,Mb N_Mb⁻¹ N_Mb,I.  The band
// factor of A = [Mt, I] (ascending band order) eliminates Mt on the way; Mb's term touches only Ib,
// the last rows of I that Mb's rows reach: it is taken from the band factor of B' = reverse([Ib, Mb])
// — Mb eliminated first, the trailing block R_II of that factor has R_IIᵀR_II = N_Ib,Ib − (Mb's
// term) — and written over A's (Ib, Ib) block before A is factored.  The sweeps of E_j = ‖R_II⁻ᵀe_j‖
// then stop at the end of I instead of running through Mb: a window's interior rows sit on average
// half a tile from that end instead of half a tile plus a margin.

// column classes of the window: 1 = A \ Ib, 2 = Ib, 3 = Mb (0: outside)
__global__ __launch_bounds__(BLOCK) void k_band_cls(int64_t n, const int32_t* __restrict__ perm, int64_t from, int8_t v,
                                                    int8_t* __restrict__ cls) {
    for (int64_t j = from + (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK)
        cls[perm[j]] = v;
}
// a live row that holds a column of A \ Ib and one of Mb couples them directly: the split is not
// exact for this Ib (err = 1)
__global__ __launch_bounds__(BLOCK) void k_band_schur_check(int64_t m, const int64_t* __restrict__ rp,
                                                            const int32_t* __restrict__ ci, const int8_t* __restrict__ cls,
                                                            const double* __restrict__ rs, int* __restrict__ err) {
    int bad = 0;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += (int64_t)gridDim.x * BLOCK) {
        if (rs[i] == 0.0) continue;
        int has = 0;
        for (int64_t f = rp[i]; f < rp[i + 1]; ++f) has |= 1 << cls[ci[f]];
        bad |= (has & 2) && (has & 8);
    }
    if (bad) atomicOr(err, 1);
}
// A's (Ib, Ib) block ← R_IIᵀR_II of B's factor, unscaled (B's positions [nm, nb) are Ib in
// descending A order: position p ↔ A position na − 1 − (p − nm)).  One workgroup per pair of B tiles
// P ≤ Q over [nm, nb); rows below nm of the first tile are masked, tiles outside B's band are 0.
__global__ __launch_bounds__(BLOCK) void k_band_schur_v(BandDev bb, const double* __restrict__ scb, int64_t nm, int64_t nb,
                                                        BandDev ba, int64_t na) {
    __shared__ double SA[TB * LDP], SB[TB * LDP];
    const int64_t K0 = nm >> 6, nt = bb.T - K0;
    // pair index -> (P, Q), P ≤ Q, both in [K0, T)
    int64_t r = blockIdx.x, P = 0;
    while (r >= nt - P) {
        r -= nt - P;
        ++P;
    }
    const int64_t Q = P + r;
    P += K0;
    const int64_t Qt = Q + K0;
    if (Qt - P > bb.w) return;   // R_KP and R_KQ never share a row inside the band: the block is 0
    d4 acc[2][2];
    acc_zero(acc);
    for (int64_t K = max<int64_t>(K0, Qt - bb.w); K <= P; ++K) {
        __syncthreads();
        const double* tp = btile(bb.R, bb.w, K, P);
        const double* tq = btile(bb.R, bb.w, K, Qt);
        for (int idx = threadIdx.x; idx < TT; idx += BLOCK) {
            const int rr = idx >> 6, c = idx & 63;
            const bool on = K * TB + rr >= nm;   // rows of eliminated (Mb) columns: not in R_II
            SA[rr * LDP + c] = on ? tp[idx] : 0.0;
            SB[rr * LDP + c] = on ? tq[idx] : 0.0;
        }
        __syncthreads();
        mma_tile<true>(SA, SB, acc);
    }
    acc_each(acc, [&](int i, int j, double v) {
        const int64_t p = P * TB + i, q = Qt * TB + j;
        if (p < nm || q < nm || p >= nb || q >= nb || p > q) return;
        const double val = v / (scb[p] * scb[q]);
        const int64_t ap = na - 1 - (p - nm), aq = na - 1 - (q - nm);   // aq ≤ ap
        btile(ba.R, ba.w, aq >> 6, ap >> 6)[(aq & 63) * TB + (ap & 63)] = val;
    });
}

// ---- many windows, pipelined (lsq_cov_band_windows) ------------------------------------------
// compute_E at scale factors hundreds of windows.  One window's factorization is a chain of T
// dependent tile steps of 1–w workgroups (latency-bound: the GPU is mostly idle), and its interior
// sweeps fill the chip only partly.  Windows are independent, so they run on NL lanes — each lane
// its own stream pair and persistent buffers (no allocation or free per window: hipFree would
// synchronise the device) — so window i + 1's factorization overlaps window i's sweeps.  The host
// waits for a lane only before reusing it.
namespace {
struct BandLane {
    hipStream_t st = nullptr, side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    DBuf<double> R, D, sc, ring, ssq, dE, dout, ev;
    DBuf<double> RB, DB, scB;       // the Schur split's bottom factor (B' = reverse([Ib, Mb]))
    DBuf<int32_t> perm, pinv, el, permB;
    DBuf<int8_t> cls;
    DBuf<int64_t> tiles, sp, segK, segE;
    DBuf<int> wmax, err;
    double *hE = nullptr, *hout = nullptr;
    int* herr = nullptr;            // [0] factor not positive definite, [1] the split's coupling check
    int64_t capE = 0, capOut = 0;
    // the window whose results are in flight on this lane
    int64_t win = -1, n = 0, nops = 0;
    double* E = nullptr;
    double* op_err = nullptr;
    const uint8_t* inner = nullptr;
    ~BandLane() {
        if (hE) (void)hipHostFree(hE);
        if (hout) (void)hipHostFree(hout);
        if (herr) (void)hipHostFree(herr);
        if (fork) (void)hipEventDestroy(fork);
        if (join) (void)hipEventDestroy(join);
        if (st) (void)hipStreamDestroy(st);
        if (side) (void)hipStreamDestroy(side);
    }
};
template <class T>
void grow(DBuf<T>& b, int64_t n) {
    if (b.n < n) b.alloc(n);
}
// results of the lane's window in flight: wait, copy out, check the factor
void lane_finish(BandLane& L) {
    if (L.win < 0) return;
    HIP_CHECK(hipStreamSynchronize(L.st));
    if (L.herr[0]) throw std::invalid_argument("lsq_cov_band_windows: AᵀA of window " + std::to_string(L.win) +
                                               " is not positive definite (rank-deficient system)");
    if (L.herr[1]) throw std::domain_error("lsq_cov_band_windows_schur: window " + std::to_string(L.win) +
                                           " has rows coupling its bottom margin to columns above Ib (a deeper Ib is needed)");
    for (int64_t j = 0; j < L.n; ++j) L.E[j] = (!L.inner || L.inner[j]) ? L.hE[j] : 0.0;
    for (int64_t i = 0; i < L.nops; ++i) L.op_err[i] = std::sqrt(L.hout[i]);
    L.win = -1;
}
}  // namespace

// ---- windows in batches: one factorization chain for several windows -----------------------------
// band_cov_windows runs one window's factorization per lane: T dependent steps of small launches
// (C4: ~1 300 steps of ~70 µs per 80-node window), so the chain's latency, not its flops, sets the
// time (round 5, serial: 93 s of factorization for 1 024 windows).  Here a lane takes LSQ_E_FBATCH
// windows at once: each window's band is assembled as before, then every step's POTRF / TRSM /
// SYRK launch serves the whole batch (band_factor_steps_batch) — first the bottom parts B' of the
// Schur split, then the A parts — and each window's sweeps follow.  Identity sweeps only (no op
// rows); the same sums as band_cov_windows, bit for bit.
namespace {
struct BatchSlot {
    DBuf<double> R, D, sc, RB, DB, scB, dE;
    DBuf<int32_t> perm, permB;
    double* hE = nullptr;
    int64_t capE = 0;
    int64_t win = -1, n = 0;
    double* E = nullptr;
    const uint8_t* inner = nullptr;
    ~BatchSlot() {
        if (hE) (void)hipHostFree(hE);
    }
};
struct BatchLane {
    hipStream_t st = nullptr, side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    DBuf<int32_t> pinv;
    DBuf<int8_t> cls;
    DBuf<int> wmax, errs, errsB;
    DBuf<double> ring, ssq;
    DBuf<int64_t> tiles;
    DBuf<BandDev> dA, dB;
    std::unique_ptr<BatchSlot[]> slots;
    std::vector<int64_t> bslot;   // the batch's B' bands: slot of each
    int* herr = nullptr;          // [0, 2·nb): A's flags per slot, [2·nb, 4·nb): B''s per B' band
    int nin = 0;
    ~BatchLane() {
        if (herr) (void)hipHostFree(herr);
        if (fork) (void)hipEventDestroy(fork);
        if (join) (void)hipEventDestroy(join);
        if (st) (void)hipStreamDestroy(st);
        if (side) (void)hipStreamDestroy(side);
    }
};
void batch_finish(BatchLane& L, int nbmax) {
    if (L.nin == 0) return;
    HIP_CHECK(hipStreamSynchronize(L.st));
    for (int i = 0; i < L.nin; ++i) {
        BatchSlot& W = L.slots[i];
        if (L.herr[2 * i]) throw std::invalid_argument("lsq_cov_band_windows: AᵀA of window " + std::to_string(W.win) +
                                                       " is not positive definite (rank-deficient system)");
        if (L.herr[2 * i + 1]) throw std::domain_error("lsq_cov_band_windows_schur: window " + std::to_string(W.win) +
                                                       " has rows coupling its bottom margin to columns above Ib (a deeper Ib is needed)");
    }
    for (size_t k = 0; k < L.bslot.size(); ++k)
        if (L.herr[2 * nbmax + 2 * k])
            throw std::invalid_argument("lsq_cov_band_windows: the bottom part of window " +
                                        std::to_string(L.slots[L.bslot[k]].win) + " is not positive definite");
    for (int i = 0; i < L.nin; ++i) {
        BatchSlot& W = L.slots[i];
        for (int64_t j = 0; j < W.n; ++j) W.E[j] = (!W.inner || W.inner[j]) ? W.hE[j] : 0.0;
        W.win = -1;
    }
    L.nin = 0;
}
// a band's width over the lane's current pinv (host readback: this lane's stream only)
int band_width_of(System& S, BatchLane& L, int64_t T) {
    L.wmax.zero(L.st);
    hipLaunchKernelGGL(k_band_width, dim3(grid_for(S.G.m)), dim3(BLOCK), 0, L.st, S.G.m, S.G.rp.p, S.G.ci.p, L.pinv.p,
                       S.rs.p, L.wmax.p);
    KERNEL_CHECK();
    int hw = 0;
    HIP_CHECK(hipMemcpyAsync(&hw, L.wmax.p, sizeof(int), hipMemcpyDeviceToHost, L.st));
    HIP_CHECK(hipStreamSynchronize(L.st));
    return (int)std::min<int64_t>(hw, T - 1);
}
// AᵀA of the columns perm[0, n) into band b (the lane's pinv set for them), equilibrated into sc
void band_assemble(System& S, BatchLane& L, const BandDev& b, int64_t n, const int32_t* perm, double* sc,
                   const BandDev* schur_from = nullptr, const double* scb = nullptr, int64_t nm = 0, int64_t nbw = 0) {
    const int64_t npad = b.T * TB;
    HIP_CHECK(hipMemsetAsync(b.R, 0, sizeof(double) * b.T * (b.w + 1) * TT, L.st));
    hipLaunchKernelGGL(k_band_normal, dim3(grid_for(npad)), dim3(BLOCK), 0, L.st, n, npad, b, perm, L.pinv.p, S.GT.rp.p,
                       S.GT.ci.p, S.GT.val.p, S.G.rp.p, S.G.ci.p, S.G.val.p, S.rs.p);
    if (schur_from) {
        const int64_t ntb = schur_from->T - (nm >> 6);
        hipLaunchKernelGGL(k_band_schur_v, dim3((unsigned)(ntb * (ntb + 1) / 2)), dim3(BLOCK), 0, L.st, *schur_from, scb,
                           nm, nbw, b, n);
    }
    hipLaunchKernelGGL(k_band_dscale, dim3(grid_for(npad)), dim3(BLOCK), 0, L.st, b, npad, sc);
    hipLaunchKernelGGL(k_band_apply_scale, dim3(grid_for(b.T * (b.w + 1) * TT)), dim3(BLOCK), 0, L.st, b, sc);
    KERNEL_CHECK();
}
}  // namespace

void band_cov_windows_batched(System& S, int64_t nwin, const int64_t* win_ptr, const int32_t* h_perm,
                              const uint8_t* inner, double* h_E, int64_t* info, const int64_t* bot_ptr,
                              const int32_t* bot_perm, const int64_t* nibs, int nbmax) {
    const int64_t ncol = S.G.n;
    const int nl = [] {
        const char* e = getenv("LSQ_E_LANES");
        return e ? std::max(1, std::min(atoi(e), 8)) : 2;
    }();
    std::vector<BatchLane> lanes(nl);
    for (BatchLane& L : lanes) {
        HIP_CHECK(hipStreamCreateWithFlags(&L.st, hipStreamNonBlocking));
        HIP_CHECK(hipStreamCreateWithFlags(&L.side, hipStreamNonBlocking));
        HIP_CHECK(hipEventCreateWithFlags(&L.fork, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&L.join, hipEventDisableTiming));
        HIP_CHECK(hipHostMalloc(&L.herr, sizeof(int) * 4 * nbmax));
        L.pinv.alloc(ncol);
        if (bot_ptr) L.cls.alloc(ncol);
        L.wmax.alloc(1);
        L.errs.alloc(2 * nbmax);
        L.errsB.alloc(2 * nbmax);
        L.dA.alloc(nbmax);
        L.dB.alloc(nbmax);
        L.slots.reset(new BatchSlot[nbmax]);
    }
    HIP_CHECK(hipStreamSynchronize(S.stream));
    int64_t products = 0, wmax_all = 0, tmax = 0, dev_bytes = 0;
    const auto t0 = std::chrono::steady_clock::now();
    try {
        int64_t batch = 0;
        for (int64_t w0 = 0; w0 < nwin; w0 += nbmax, ++batch) {
            BatchLane& L = lanes[batch % nl];
            batch_finish(L, nbmax);
            const int nb = (int)std::min<int64_t>(nbmax, nwin - w0);
            hipStream_t st = L.st;
            L.errs.zero(st);
            L.errsB.zero(st);
            // 1. the bottom parts B' (Schur split), then their factorization as one batch
            std::vector<BandDev> hb, ha(nb);
            std::vector<int64_t> nms(nb, 0), nbws(nb, 0);
            std::vector<int> bidx(nb, -1);
            L.bslot.clear();
            for (int i = 0; i < nb; ++i) {
                const int64_t w = w0 + i, n = win_ptr[w + 1] - win_ptr[w];
                BatchSlot& W = L.slots[i];
                const int64_t nbw = bot_ptr ? bot_ptr[w + 1] - bot_ptr[w] : 0, nib = nbw > 0 ? nibs[w] : 0;
                if (nbw > 0 && (nib < 1 || nbw - nib < 1 || nib > n))
                    throw std::invalid_argument("lsq_cov_band_windows_schur: bad bottom part of window " + std::to_string(w));
                nbws[i] = nbw;
                nms[i] = nbw - nib;
                if (nbw == 0) continue;
                const int64_t TBb = (nbw + TB - 1) / TB;
                grow(W.permB, nbw);
                W.permB.upload(bot_perm + bot_ptr[w], nbw, st);
                HIP_CHECK(hipMemsetAsync(L.pinv.p, 0xff, sizeof(int32_t) * ncol, st));
                hipLaunchKernelGGL(k_band_pinv, dim3(grid_for(nbw)), dim3(BLOCK), 0, st, nbw, W.permB.p, L.pinv.p);
                const int bwb = band_width_of(S, L, TBb);
                grow(W.RB, TBb * (int64_t)(bwb + 1) * TT);
                grow(W.DB, TBb * TT);
                grow(W.scB, TBb * TB);
                const BandDev bB{TBb, bwb, W.RB.p, W.DB.p};
                band_assemble(S, L, bB, nbw, W.permB.p, W.scB.p);
                bidx[i] = (int)hb.size();
                hb.push_back(bB);
                L.bslot.push_back(i);
            }
            if (!hb.empty()) {
                L.dB.upload(hb.data(), (int64_t)hb.size(), st);
                band_factor_steps_batch(L.dB.p, hb, st, L.side, L.fork, L.join, L.errsB.p);
            }
            // 2. the A parts: the split's coupling check, AᵀA with the Schur block, one factorization
            for (int i = 0; i < nb; ++i) {
                const int64_t w = w0 + i, n = win_ptr[w + 1] - win_ptr[w], T = (n + TB - 1) / TB;
                BatchSlot& W = L.slots[i];
                grow(W.perm, n);
                W.perm.upload(h_perm + win_ptr[w], n, st);
                const int64_t nbw = nbws[i], nm = nms[i], nib = nbw - nm;
                if (nbw > 0) {
                    HIP_CHECK(hipMemsetAsync(L.cls.p, 0, ncol, st));
                    hipLaunchKernelGGL(k_band_cls, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, W.perm.p, (int64_t)0,
                                       (int8_t)1, L.cls.p);
                    hipLaunchKernelGGL(k_band_cls, dim3(grid_for(nib)), dim3(BLOCK), 0, st, n, W.perm.p, n - nib,
                                       (int8_t)2, L.cls.p);
                    hipLaunchKernelGGL(k_band_cls, dim3(grid_for(nm)), dim3(BLOCK), 0, st, nm, W.permB.p, (int64_t)0,
                                       (int8_t)3, L.cls.p);
                    hipLaunchKernelGGL(k_band_schur_check, dim3(grid_for(S.G.m)), dim3(BLOCK), 0, st, S.G.m, S.G.rp.p,
                                       S.G.ci.p, L.cls.p, S.rs.p, L.errs.p + 2 * i + 1);
                    KERNEL_CHECK();
                }
                HIP_CHECK(hipMemsetAsync(L.pinv.p, 0xff, sizeof(int32_t) * ncol, st));
                hipLaunchKernelGGL(k_band_pinv, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, W.perm.p, L.pinv.p);
                int bw = band_width_of(S, L, T);
                if (nbw > 0) bw = (int)std::min<int64_t>(std::max<int64_t>(bw, ((n - 1) >> 6) - ((n - nib) >> 6)), T - 1);
                grow(W.R, T * (int64_t)(bw + 1) * TT);
                grow(W.D, T * TT);
                grow(W.sc, T * TB);
                grow(W.dE, n);
                ha[i] = BandDev{T, bw, W.R.p, W.D.p};
                if (nbw > 0) band_assemble(S, L, ha[i], n, W.perm.p, W.sc.p, &hb[bidx[i]], W.scB.p, nm, nbw);
                else band_assemble(S, L, ha[i], n, W.perm.p, W.sc.p);
                wmax_all = std::max<int64_t>(wmax_all, bw);
                tmax = std::max(tmax, T);
            }
            L.dA.upload(ha.data(), nb, st);
            band_factor_steps_batch(L.dA.p, ha, st, L.side, L.fork, L.join, L.errs.p);
            // 3. each window's sweeps over the tiles holding an inner position
            for (int i = 0; i < nb; ++i) {
                const int64_t w = w0 + i, n = win_ptr[w + 1] - win_ptr[w], T = ha[i].T;
                const uint8_t* inw = inner ? inner + win_ptr[w] : nullptr;
                BatchSlot& W = L.slots[i];
                std::vector<int64_t> tiles;
                for (int64_t J = 0; J < T; ++J) {
                    bool any = !inw;
                    for (int64_t j = J * TB; j < std::min<int64_t>(n, (J + 1) * TB) && !any; ++j) any = inw[j] != 0;
                    if (any) tiles.push_back(J);
                }
                const int64_t nsw = (int64_t)tiles.size(), ring_wg = (int64_t)(ha[i].w + 1) * TT;
                for (int64_t J : tiles) products += (T - J) * (int64_t)std::min<int64_t>(ha[i].w + 1, T - J);
                int64_t cap = std::max<int64_t>(nsw, 1);
                if (L.ring.n < cap * ring_wg) {
                    size_t free_b = 0, total_b = 0;
                    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
                    const double room = 0.8 * (double)free_b + (double)L.ring.n * sizeof(double);
                    cap = std::min<int64_t>(cap, (int64_t)(room / ((double)ring_wg * sizeof(double))));
                    if (cap < 1) throw Refused("lsq_cov_band_windows: no device memory left for a window's sweeps");
                    if (L.ring.n < cap * ring_wg) L.ring.alloc(cap * ring_wg);
                }
                cap = std::min<int64_t>(std::max<int64_t>(nsw, 1), L.ring.n / ring_wg);
                grow(L.ssq, T * TB);
                HIP_CHECK(hipMemsetAsync(L.ssq.p, 0, sizeof(double) * T * TB, st));
                if (nsw > 0) {
                    grow(L.tiles, nsw);
                    L.tiles.upload(tiles.data(), nsw, st);
                    run_sweeps<true>(st, ha[i], nsw, cap, L.tiles.p, nullptr, nullptr, nullptr, nullptr, W.sc.p, L.ring.p,
                                     L.ssq.p);
                }
                hipLaunchKernelGGL(k_band_diag_sweep, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, nullptr, L.ssq.p, W.sc.p,
                                   W.dE.p);
                KERNEL_CHECK();
                if (W.capE < n) {
                    if (W.hE) HIP_CHECK(hipHostFree(W.hE));
                    HIP_CHECK(hipHostMalloc(&W.hE, sizeof(double) * n));
                    W.capE = n;
                }
                HIP_CHECK(hipMemcpyAsync(W.hE, W.dE.p, sizeof(double) * n, hipMemcpyDeviceToHost, st));
                W.win = w;
                W.n = n;
                W.E = h_E + win_ptr[w];
                W.inner = inw;
                dev_bytes = std::max<int64_t>(dev_bytes, (int64_t)(W.R.n + W.RB.n) * (int64_t)sizeof(double));
            }
            HIP_CHECK(hipMemcpyAsync(L.herr, L.errs.p, sizeof(int) * 2 * nb, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipMemcpyAsync(L.herr + 2 * nbmax, L.errsB.p, sizeof(int) * 2 * nbmax, hipMemcpyDeviceToHost, st));
            L.nin = nb;
        }
        for (BatchLane& L : lanes) batch_finish(L, nbmax);
    } catch (...) {
        for (BatchLane& L : lanes)
            if (L.st) (void)hipStreamSynchronize(L.st);
        throw;
    }
    if (info) {
        info[0] = wmax_all;
        info[1] = tmax;
        info[2] = dev_bytes * nbmax * nl;
        info[3] = products;
        info[4] = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
        info[5] = nl;
    }
}

void band_cov_windows(System& S, int64_t nwin, const int64_t* win_ptr, const int32_t* h_perm, const uint8_t* inner,
                      double* h_E, const int64_t* win_ops, const int64_t* op_ptr, const int32_t* op_pos,
                      const double* op_val, double* op_err, int64_t* info, const int64_t* bot_ptr,
                      const int32_t* bot_perm, const int64_t* nibs) {
    refresh_scaling(S, S.cs_mode < 0 ? 0 : S.cs_mode);
    ensure_full_csr(S);   // the band of AᵀA from G / GT
    const int64_t ncol = S.G.n;
    int64_t nmax = 0, omax = 0;
    for (int64_t w = 0; w < nwin; ++w) {
        const int64_t n = win_ptr[w + 1] - win_ptr[w];
        if (n < 1 || n > ncol) throw std::invalid_argument("lsq_cov_band_windows: bad window");
        nmax = std::max(nmax, n);
        if (win_ops) omax = std::max(omax, win_ops[w + 1] - win_ops[w]);
        for (int64_t j = win_ptr[w]; j < win_ptr[w + 1]; ++j)
            if (h_perm[j] < 0 || h_perm[j] >= ncol) throw std::invalid_argument("lsq_cov_band_windows: column out of range");
        if (win_ops)
            for (int64_t i = win_ops[w]; i < win_ops[w + 1]; ++i)
                for (int64_t e = op_ptr[i]; e < op_ptr[i + 1]; ++e)
                    if (op_pos[e] < 0 || op_pos[e] >= n)
                        throw std::invalid_argument("lsq_cov_band_windows: an op row reaches outside its window");
    }
    static const int fbatch = getenv("LSQ_E_FBATCH") ? std::max(1, std::min(atoi(getenv("LSQ_E_FBATCH")), 32)) : 8;
    if (!win_ops && fbatch > 1 && nwin > 1) {   // identity sweeps only: windows in batches
        band_cov_windows_batched(S, nwin, win_ptr, h_perm, inner, h_E, info, bot_ptr, bot_perm, nibs,
                                 (int)std::min<int64_t>(fbatch, nwin));
        return;
    }
    const int nl = [] {
        const char* e = getenv("LSQ_E_LANES");
        return e ? std::max(1, std::min(atoi(e), 8)) : 2;   // C4, 32-node tiles: 2 lanes 132 s, 4 lanes 134 s
    }();
    std::vector<BandLane> lanes(nl);
    const int64_t nopad = (omax + TB - 1) / TB * TB;
    for (BandLane& L : lanes) {
        HIP_CHECK(hipStreamCreateWithFlags(&L.st, hipStreamNonBlocking));
        HIP_CHECK(hipStreamCreateWithFlags(&L.side, hipStreamNonBlocking));
        HIP_CHECK(hipEventCreateWithFlags(&L.fork, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&L.join, hipEventDisableTiming));
        HIP_CHECK(hipHostMalloc(&L.hE, sizeof(double) * std::max<int64_t>(nmax, 1)));
        HIP_CHECK(hipHostMalloc(&L.hout, sizeof(double) * std::max<int64_t>(nopad, 1)));
        HIP_CHECK(hipHostMalloc(&L.herr, 2 * sizeof(int)));
        L.pinv.alloc(ncol);
        L.wmax.alloc(1);
        L.err.alloc(2);
        if (bot_ptr) L.cls.alloc(ncol);
    }
    HIP_CHECK(hipStreamSynchronize(S.stream));   // formation / scaling done before the lanes read them
    int64_t products = 0, wmax_all = 0, tmax = 0, dev_bytes = 0;
    const auto t0 = std::chrono::steady_clock::now();
    try {
        for (int64_t w = 0; w < nwin; ++w) {
            BandLane& L = lanes[w % nl];
            lane_finish(L);
            const int64_t n = win_ptr[w + 1] - win_ptr[w], T = (n + TB - 1) / TB, npad = T * TB;
            const int32_t* perm = h_perm + win_ptr[w];
            const uint8_t* inw = inner ? inner + win_ptr[w] : nullptr;
            hipStream_t st = L.st;
            L.err.zero(st);
            // the Schur split (bot_ptr): B' = reverse([Ib, Mb]) factored first; its trailing Ib block
            // replaces A's (Ib, Ib) block below
            const int64_t nbw = bot_ptr ? bot_ptr[w + 1] - bot_ptr[w] : 0, nib = nbw > 0 ? nibs[w] : 0, nm = nbw - nib;
            if (nbw > 0 && (nib < 1 || nm < 1 || nib > n))
                throw std::invalid_argument("lsq_cov_band_windows_schur: bad bottom part of window " + std::to_string(w));
            BandDev bB{0, 0, nullptr, nullptr};
            if (nbw > 0) {
                const int64_t TBb = (nbw + TB - 1) / TB, npb = TBb * TB;
                grow(L.permB, nbw);
                L.permB.upload(bot_perm + bot_ptr[w], nbw, st);
                HIP_CHECK(hipMemsetAsync(L.pinv.p, 0xff, sizeof(int32_t) * ncol, st));
                hipLaunchKernelGGL(k_band_pinv, dim3(grid_for(nbw)), dim3(BLOCK), 0, st, nbw, L.permB.p, L.pinv.p);
                L.wmax.zero(st);
                hipLaunchKernelGGL(k_band_width, dim3(grid_for(S.G.m)), dim3(BLOCK), 0, st, S.G.m, S.G.rp.p, S.G.ci.p,
                                   L.pinv.p, S.rs.p, L.wmax.p);
                KERNEL_CHECK();
                int hwb = 0;
                HIP_CHECK(hipMemcpyAsync(&hwb, L.wmax.p, sizeof(int), hipMemcpyDeviceToHost, st));
                HIP_CHECK(hipStreamSynchronize(st));
                const int bwb = (int)std::min<int64_t>(hwb, TBb - 1);
                grow(L.RB, TBb * (int64_t)(bwb + 1) * TT);
                grow(L.DB, TBb * TT);
                grow(L.scB, npb);
                bB = BandDev{TBb, bwb, L.RB.p, L.DB.p};
                HIP_CHECK(hipMemsetAsync(L.RB.p, 0, sizeof(double) * TBb * (bwb + 1) * TT, st));
                hipLaunchKernelGGL(k_band_normal, dim3(grid_for(npb)), dim3(BLOCK), 0, st, nbw, npb, bB, L.permB.p,
                                   L.pinv.p, S.GT.rp.p, S.GT.ci.p, S.GT.val.p, S.G.rp.p, S.G.ci.p, S.G.val.p, S.rs.p);
                hipLaunchKernelGGL(k_band_dscale, dim3(grid_for(npb)), dim3(BLOCK), 0, st, bB, npb, L.scB.p);
                hipLaunchKernelGGL(k_band_apply_scale, dim3(grid_for(TBb * (bwb + 1) * TT)), dim3(BLOCK), 0, st, bB,
                                   L.scB.p);
                KERNEL_CHECK();
                band_factor_steps(bB, st, L.side, L.fork, L.join, L.err.p);
            }
            // the window's order on the device and its inverse over every compact column (−1 outside)
            grow(L.perm, n);
            L.perm.upload(perm, n, st);
            if (nbw > 0) {   // exactness of the split: no live row holds a column of A \ Ib and one of Mb
                HIP_CHECK(hipMemsetAsync(L.cls.p, 0, ncol, st));
                hipLaunchKernelGGL(k_band_cls, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, L.perm.p, (int64_t)0, (int8_t)1,
                                   L.cls.p);
                hipLaunchKernelGGL(k_band_cls, dim3(grid_for(nib)), dim3(BLOCK), 0, st, n, L.perm.p, n - nib, (int8_t)2,
                                   L.cls.p);
                hipLaunchKernelGGL(k_band_cls, dim3(grid_for(nm)), dim3(BLOCK), 0, st, nm, L.permB.p, (int64_t)0,
                                   (int8_t)3, L.cls.p);
                hipLaunchKernelGGL(k_band_schur_check, dim3(grid_for(S.G.m)), dim3(BLOCK), 0, st, S.G.m, S.G.rp.p,
                                   S.G.ci.p, L.cls.p, S.rs.p, L.err.p + 1);
                KERNEL_CHECK();
            }
            HIP_CHECK(hipMemsetAsync(L.pinv.p, 0xff, sizeof(int32_t) * ncol, st));
            hipLaunchKernelGGL(k_band_pinv, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, L.perm.p, L.pinv.p);
            L.wmax.zero(st);
            hipLaunchKernelGGL(k_band_width, dim3(grid_for(S.G.m)), dim3(BLOCK), 0, st, S.G.m, S.G.rp.p, S.G.ci.p,
                               L.pinv.p, S.rs.p, L.wmax.p);
            KERNEL_CHECK();
            int hw = 0;
            HIP_CHECK(hipMemcpyAsync(&hw, L.wmax.p, sizeof(int), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));   // this lane only: the others keep running
            int bw = (int)std::min<int64_t>(hw, T - 1);
            if (nbw > 0)   // A's band holds the dense (Ib, Ib) block the split writes
                bw = (int)std::min<int64_t>(std::max<int64_t>(bw, ((n - 1) >> 6) - ((n - nib) >> 6)), T - 1);
            const int64_t band_tiles = T * (int64_t)(bw + 1);
            // the interior's tiles (the sweeps) and the op rows' sweep plan (positions: no pinv)
            std::vector<int64_t> tiles;
            for (int64_t J = 0; J < T; ++J) {
                bool any = !inw;
                for (int64_t j = J * TB; j < std::min<int64_t>(n, (J + 1) * TB) && !any; ++j) any = inw[j] != 0;
                if (any) tiles.push_back(J);
            }
            const int64_t nops = win_ops ? win_ops[w + 1] - win_ops[w] : 0;
            SweepOps so;
            if (nops > 0) {
                std::vector<int64_t> rows(nops);
                for (int64_t i = 0; i < nops; ++i) rows[i] = win_ops[w] + i;
                so = sweep_ops(rows, op_ptr, op_pos, op_val, nullptr, T, bw);
            }
            const int64_t nsw = (int64_t)tiles.size(), nopw = nops > 0 ? (int64_t)so.sp.size() - 1 : 0;
            for (int64_t J : tiles) products += (T - J) * (int64_t)std::min<int64_t>(bw + 1, T - J);
            products += so.gemms;
            // sweep rings for up to `cap` concurrent workgroups (run_sweeps batches the rest): every
            // tile of the interior at once when the device has the room, else as many as fit the
            // free memory (band_cov's rule) — a wide band then sweeps in batches instead of failing
            const int64_t want = std::max<int64_t>({nsw, nopw, 1}), ring_wg = (int64_t)(bw + 1) * TT;
            int64_t cap = want;
            if (L.R.n < band_tiles * TT || L.D.n < T * TT || L.ring.n < want * ring_wg) {
                size_t free_b = 0, total_b = 0;
                HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
                const double grow_rd = (double)(std::max<int64_t>(band_tiles * TT - L.R.n, 0) +
                                                std::max<int64_t>(T * TT - L.D.n, 0)) * sizeof(double);
                const double room = 0.8 * (double)free_b + (double)L.ring.n * sizeof(double) - grow_rd;
                cap = std::min<int64_t>(want, (int64_t)(room / ((double)ring_wg * sizeof(double))));
                if (cap < 1)
                    throw Refused("lsq_cov_band_windows: a window band of " + std::to_string(bw) +
                                  " tiles needs " + std::to_string((int64_t)grow_rd >> 20) +
                                  " MiB more, more than the device has free (fewer lanes: LSQ_E_LANES)");
            }
            const int64_t need = (band_tiles + T + cap * (bw + 1)) * TT * (int64_t)sizeof(double);
            grow(L.R, band_tiles * TT);
            grow(L.D, T * TT);
            grow(L.sc, npad);
            grow(L.ssq, npad);
            grow(L.dE, n);
            grow(L.ring, cap * (bw + 1) * TT);
            dev_bytes = std::max<int64_t>(dev_bytes, nl * need);
            wmax_all = std::max<int64_t>(wmax_all, bw);
            tmax = std::max(tmax, T);
            HIP_CHECK(hipMemsetAsync(L.R.p, 0, sizeof(double) * band_tiles * TT, st));
            BandDev b{T, bw, L.R.p, L.D.p};
            hipLaunchKernelGGL(k_band_normal, dim3(grid_for(npad)), dim3(BLOCK), 0, st, n, npad, b, L.perm.p, L.pinv.p,
                               S.GT.rp.p, S.GT.ci.p, S.GT.val.p, S.G.rp.p, S.G.ci.p, S.G.val.p, S.rs.p);
            if (nbw > 0) {   // (Ib, Ib) ← N_Ib,Ib − N_Ib,Mb N_Mb⁻¹ N_Mb,Ib from B's factor
                const int64_t ntb = bB.T - (nm >> 6);
                hipLaunchKernelGGL(k_band_schur_v, dim3((unsigned)(ntb * (ntb + 1) / 2)), dim3(BLOCK), 0, st, bB, L.scB.p,
                                   nm, nbw, b, n);
                KERNEL_CHECK();
            }
            hipLaunchKernelGGL(k_band_dscale, dim3(grid_for(npad)), dim3(BLOCK), 0, st, b, npad, L.sc.p);
            hipLaunchKernelGGL(k_band_apply_scale, dim3(grid_for(band_tiles * TT)), dim3(BLOCK), 0, st, b, L.sc.p);
            KERNEL_CHECK();
            band_factor_steps(b, st, L.side, L.fork, L.join, L.err.p);
            HIP_CHECK(hipMemcpyAsync(L.herr, L.err.p, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
            // the diagonal over the interior's tiles, E in window order
            HIP_CHECK(hipMemsetAsync(L.ssq.p, 0, sizeof(double) * npad, st));
            if (nsw > 0) {
                grow(L.tiles, nsw);
                L.tiles.upload(tiles.data(), nsw, st);
                run_sweeps<true>(st, b, nsw, cap, L.tiles.p, nullptr, nullptr, nullptr, nullptr, L.sc.p, L.ring.p,
                                 L.ssq.p);
            }
            hipLaunchKernelGGL(k_band_diag_sweep, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, nullptr, L.ssq.p, L.sc.p,
                               L.dE.p);
            KERNEL_CHECK();
            HIP_CHECK(hipMemcpyAsync(L.hE, L.dE.p, sizeof(double) * n, hipMemcpyDeviceToHost, st));
            if (nops > 0) {   // the op rows' errors
                grow(L.sp, nopw + 1);
                grow(L.segK, (int64_t)so.segK.size());
                grow(L.segE, (int64_t)so.segE.size());
                grow(L.el, std::max<int64_t>((int64_t)so.el.size(), 1));
                grow(L.ev, std::max<int64_t>((int64_t)so.ev.size(), 1));
                grow(L.dout, nopw * TB);
                L.sp.upload(so.sp.data(), nopw + 1, st);
                L.segK.upload(so.segK.data(), (int64_t)so.segK.size(), st);
                L.segE.upload(so.segE.data(), (int64_t)so.segE.size(), st);
                L.el.upload(so.el.data(), (int64_t)so.el.size(), st);
                L.ev.upload(so.ev.data(), (int64_t)so.ev.size(), st);
                run_sweeps<false>(st, b, nopw, cap, L.sp.p, L.segK.p, L.segE.p, L.el.p, L.ev.p, L.sc.p, L.ring.p,
                                  L.dout.p);
                HIP_CHECK(hipMemcpyAsync(L.hout, L.dout.p, sizeof(double) * nops, hipMemcpyDeviceToHost, st));
            }
            L.win = w;
            L.n = n;
            L.nops = nops;
            L.E = h_E + win_ptr[w];
            L.op_err = nops > 0 ? op_err + win_ops[w] : nullptr;
            L.inner = inw;
        }
        for (BandLane& L : lanes) lane_finish(L);
    } catch (...) {
        for (BandLane& L : lanes)
            if (L.st) (void)hipStreamSynchronize(L.st);
        throw;
    }
    if (info) {
        info[0] = wmax_all;
        info[1] = tmax;
        info[2] = dev_bytes;
        info[3] = products;
        info[4] = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
        info[5] = nl;
    }
}

}  // namespace lsq
