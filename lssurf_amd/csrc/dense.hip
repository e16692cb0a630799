// dense.hip — device dense factorisation for small / ill-conditioned systems (n ≲ 40 k).
//
//   N = AᵀA (upper triangle, deterministic: one thread owns one row of N)
//   N = RᵀR           blocked right-looking Cholesky, 64x64 tiles: POTRF (1 WG, LDS) → TRSM
//                     panel (1 WG per block column) → SYRK/GEMM trailing update (1 WG per tile)
//   R⁻¹               blocked TRTRI, bottom block row first: D = R_ii⁻¹ (LDS), then every
//                     R⁻¹_ij = −D Σ_k R_ik R⁻¹_kj as one 64x64 tile per workgroup
//
// R⁻¹ is (1) an exact right preconditioner for LSQR (A R⁻¹ has condition ~1, so LSQR converges
// in a handful of iterations even when column scaling would need ~50 k), and (2) the factor
// the reference's error propagation inverts (smooth_fit.py:218-253: rz → inv_tr_upper →
// sqrt(row sums of R⁻¹²) = sqrt(diag((AᵀA)⁻¹))).  The matrices are npad x npad row-major
// (npad = n rounded up to 64, identity on the padding) in HBM.
#include <cmath>

#include "system.hpp"

namespace lsq {
namespace {

constexpr int TB = 64;          // tile edge
constexpr int LDP = TB + 1;     // LDS row pitch (bank-conflict padding)

__global__ __launch_bounds__(BLOCK) void k_normal_rows(int64_t n, int64_t npad, int64_t ld,
                                                       const int64_t* __restrict__ trp, const int32_t* __restrict__ tci,
                                                       const double* __restrict__ tval, const int64_t* __restrict__ rp,
                                                       const int32_t* __restrict__ ci, const double* __restrict__ val,
                                                       const double* __restrict__ rs, double* __restrict__ Nm) {
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < npad; j += (int64_t)gridDim.x * BLOCK) {
        double* row = Nm + j * ld;
        if (j >= n) {
            row[j] = 1.0;
            continue;
        }
        for (int64_t e = trp[j]; e < trp[j + 1]; ++e) {
            const int32_t i = tci[e];
            const double a = tval[e] * rs[i];
            if (a == 0.0) continue;
            for (int64_t f = rp[i]; f < rp[i + 1]; ++f) {
                const int32_t k = ci[f];
                if (k < j) continue;
                row[k] += a * (val[f] * rs[i]);
            }
        }
    }
}

// The three sequential tile kernels of the chain (POTRF, TRSM panel, TRTRI diagonal) run as ONE
// wave with lane c owning column c of the tile in registers: no workgroup barriers on the 64
// dependent steps (the 256-thread LDS versions waited on 2–3 barriers per step: 88 / 82 / 45 µs
// per tile).  The arithmetic is the same expressions in the same order.
constexpr int TW = 64;   // threads per tile kernel (one wave)

// lane l's copy of v (l uniform): two v_readlane into SGPRs, no LDS round trip
__device__ __forceinline__ double lane_bcast(double v, int l) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Cholesky of the diagonal tile (upper).  err[0] set if a pivot is not positive (the pivot is
// then taken as 1).  Lane c holds A[0..63][c]; A[j][i] (i > j) is lane i's a[j].
__global__ __launch_bounds__(TW) void k_potrf_diag(double* __restrict__ Nm, int64_t ld, int64_t k0, int* err) {
    const int c = threadIdx.x;
    double a[TB];
#pragma unroll
    for (int r = 0; r < TB; ++r) a[r] = c >= r ? Nm[(k0 + r) * ld + k0 + c] : 0.0;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < TB; ++j) {
        const double d = lane_bcast(a[j], j);
        const bool ok = d > 0.0;
        bad |= !ok;
        const double piv = ok ? sqrt(d) : 1.0;
        a[j] = c == j ? piv : a[j] / piv;
#pragma unroll
        for (int i = j + 1; i < TB; ++i) a[i] -= lane_bcast(a[j], i) * a[j];
    }
    if (bad && c == 0) atomicExch(err, 1);
#pragma unroll
    for (int r = 0; r < TB; ++r)
        if (c >= r) Nm[(k0 + r) * ld + k0 + c] = a[r];
}

// Panel: X = R_kk^{-T} N[k0:k0+64, j0:j0+64] for every block column right of the diagonal.
// Lane c holds column c of X; R_kk's rows are read from LDS at one address per wave (broadcast).
__global__ __launch_bounds__(TW) void k_trsm_panel(double* __restrict__ Nm, int64_t ld, int64_t k0) {
    __shared__ double R[TB * TB];
    const int c = threadIdx.x;
    const int64_t j0 = k0 + (int64_t)(blockIdx.x + 1) * TB;
    double x[TB];
#pragma unroll
    for (int r = 0; r < TB; ++r) {
        R[r * TB + c] = Nm[(k0 + r) * ld + k0 + c];
        x[r] = Nm[(k0 + r) * ld + j0 + c];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TB; ++i) {
        x[i] /= R[i * TB + i];
#pragma unroll
        for (int p = i + 1; p < TB; ++p) x[p] -= R[i * TB + p] * x[i];
    }
#pragma unroll
    for (int r = 0; r < TB; ++r) Nm[(k0 + r) * ld + j0 + c] = x[r];
}

// Trailing update of upper tiles (ib <= jb): N[ib, jb] -= P[:, ib]ᵀ P[:, jb], P = panel rows.
__global__ __launch_bounds__(BLOCK) void k_syrk_tiles(double* __restrict__ Nm, int64_t ld, int64_t k0, int m) {
    const int ib = blockIdx.x % m, jb = blockIdx.x / m;
    if (jb < ib) return;
    __shared__ double Pi[TB * LDP];
    __shared__ double Pj[TB * LDP];
    const int64_t c0 = k0 + TB + (int64_t)ib * TB, d0 = k0 + TB + (int64_t)jb * TB;
    for (int idx = threadIdx.x; idx < TB * TB; idx += BLOCK) {
        const int p = idx / TB, c = idx % TB;
        Pi[p * LDP + c] = Nm[(k0 + p) * ld + c0 + c];
        Pj[p * LDP + c] = Nm[(k0 + p) * ld + d0 + c];
    }
    __syncthreads();
    const int tr = threadIdx.x / 16, tc = threadIdx.x % 16;
    double acc[4][4] = {};
    for (int p = 0; p < TB; ++p) {
        double a[4], b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a[q] = Pi[p * LDP + tr * 4 + q];
            b[q] = Pj[p * LDP + tc * 4 + q];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int s = 0; s < 4; ++s) acc[q][s] += a[q] * b[s];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int s = 0; s < 4; ++s) Nm[(c0 + tr * 4 + q) * ld + d0 + tc * 4 + s] -= acc[q][s];
}

// Inverse of the upper-triangular diagonal tile R_ii into Ri_ii: lane c back-substitutes column c
// (x_j = 0 for j > c, so the sums over j ≤ 63 add exact zeros past c and rows i > c come out 0).
__global__ __launch_bounds__(TW) void k_trinv_diag(const double* __restrict__ R, double* __restrict__ Ri,
                                                   int64_t ld, int64_t i0) {
    __shared__ double A[TB * TB];
    const int c = threadIdx.x;
#pragma unroll
    for (int r = 0; r < TB; ++r) A[r * TB + c] = c >= r ? R[(i0 + r) * ld + i0 + c] : 0.0;
    __syncthreads();
    double x[TB];
#pragma unroll
    for (int i = TB - 1; i >= 0; --i) {
        double xi = i == c ? 1.0 : 0.0;
#pragma unroll
        for (int j = i + 1; j < TB; ++j) xi -= A[i * TB + j] * x[j];
        x[i] = xi / A[i * TB + i];
    }
#pragma unroll
    for (int r = 0; r < TB; ++r) Ri[(i0 + r) * ld + i0 + c] = x[r];
}

// Ri[ib, jb] = −Ri_ii · Σ_{kb=ib+1..jb} R[ib, kb] · Ri[kb, jb]   for jb = ib+1+blockIdx.x
__global__ __launch_bounds__(BLOCK) void k_trinv_row(const double* __restrict__ R, double* __restrict__ Ri, int64_t ld,
                                                     int ib) {
    const int jb = ib + 1 + blockIdx.x;
    __shared__ double Ta[TB * LDP];
    __shared__ double Tb[TB * LDP];
    const int tr = threadIdx.x / 16, tc = threadIdx.x % 16;
    double acc[4][4] = {};
    const int64_t r0 = (int64_t)ib * TB, c0 = (int64_t)jb * TB;
    for (int kb = ib + 1; kb <= jb; ++kb) {
        const int64_t k0 = (int64_t)kb * TB;
        __syncthreads();
        for (int idx = threadIdx.x; idx < TB * TB; idx += BLOCK) {
            const int r = idx / TB, c = idx % TB;
            Ta[r * LDP + c] = R[(r0 + r) * ld + k0 + c];     // R[ib, kb]   (rows r, inner c)
            Tb[r * LDP + c] = Ri[(k0 + r) * ld + c0 + c];    // Ri[kb, jb]  (inner r, cols c)
        }
        __syncthreads();
        for (int p = 0; p < TB; ++p) {
            double a[4], b[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a[q] = Ta[(tr * 4 + q) * LDP + p];
                b[q] = Tb[p * LDP + tc * 4 + q];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int s = 0; s < 4; ++s) acc[q][s] += a[q] * b[s];
        }
    }
    // T -> LDS, then multiply by −Ri_ii
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int s = 0; s < 4; ++s) Tb[(tr * 4 + q) * LDP + tc * 4 + s] = acc[q][s];
    for (int idx = threadIdx.x; idx < TB * TB; idx += BLOCK) {
        const int r = idx / TB, c = idx % TB;
        Ta[r * LDP + c] = Ri[(r0 + r) * ld + r0 + c];
    }
    __syncthreads();
    double out[4][4] = {};
    for (int p = 0; p < TB; ++p) {
        double a[4], b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a[q] = Ta[(tr * 4 + q) * LDP + p];
            b[q] = Tb[p * LDP + tc * 4 + q];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int s = 0; s < 4; ++s) out[q][s] += a[q] * b[s];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int s = 0; s < 4; ++s) Ri[(r0 + tr * 4 + q) * ld + c0 + tc * 4 + s] = -out[q][s];
}

__global__ __launch_bounds__(BLOCK) void k_zero_lower(double* __restrict__ M, int64_t npad, int64_t ld) {
    for (int64_t idx = (int64_t)blockIdx.x * BLOCK + threadIdx.x; idx < npad * npad;
         idx += (int64_t)gridDim.x * BLOCK) {
        const int64_t r = idx / npad, c = idx % npad;
        if (c < r) M[r * ld + c] = 0.0;
    }
}

// E_i = sqrt(Σ_{k >= i} Ri[i][k]²), summed k descending (propagate_qz_errors order)
__global__ __launch_bounds__(BLOCK) void k_rowrss_dense(const double* __restrict__ Ri, int64_t n, int64_t ld,
                                                        double* __restrict__ E) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    // lanes take interleaved columns; partial sums combined in a fixed tree: deterministic
    double s = 0.0;
    for (int64_t k = n - 1 - lane; k >= i; k -= 64) {
        const double x = Ri[i * ld + k];
        s += x * x;
    }
    s = wave_sum(s);
    if (lane == 0) E[i] = sqrt(s);
}

}  // namespace

// ---- GEMV kernels used inside the preconditioned LSQR (exported to lsqr.hip) ---------------
// z_i = scale · Σ_{j >= i} M[i][j] v_j   (upper-triangular M, one wave per row)
__global__ __launch_bounds__(BLOCK) void k_gemv_upper(const double* __restrict__ M, int64_t n, int64_t ld,
                                                      const double* __restrict__ v, const LsqState* __restrict__ st,
                                                      int scale_mode, double* __restrict__ z) {
    if (st && st->stop && scale_mode != 2) return;
    const int lane = threadIdx.x & 63;
    const double scale = scale_mode == 1 ? st->inv_alpha : 1.0;
    for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (int64_t)gridDim.x * 4) {
        double s = 0.0;
        for (int64_t j = i + lane; j < n; j += 64) s += M[i * ld + j] * v[j];
        s = wave_sum(s);
        if (lane == 0) z[i] = s * scale;
    }
}

// out_j = Σ_{i <= j} M[i][j] t_i  (= (Mᵀ t)_j), one thread per column, coalesced along rows;
// epilogue (mode 1): out = out·(1/β) − β·vin·(1/α), partial Σout²
__global__ __launch_bounds__(BLOCK) void k_gemvT_upper(const double* __restrict__ M, int64_t n, int64_t ld,
                                                       const double* __restrict__ t, const LsqState* __restrict__ st,
                                                       int mode, const double* __restrict__ vin,
                                                       double* __restrict__ out, double* part) {
    if (st && st->stop) return;
    double sv = 0.0;
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK) {
        double a0 = 0.0, a1 = 0.0;
        int64_t i = 0;
        for (; i + 1 <= j; i += 2) {
            a0 += M[i * ld + j] * t[i];
            a1 += M[(i + 1) * ld + j] * t[i + 1];
        }
        if (i <= j) a0 += M[i * ld + j] * t[i];
        double o = a0 + a1;
        if (mode == 1) {
            if (st->skip_v) o = vin[j];
            else o = o * st->inv_beta - st->beta * (vin[j] * st->inv_alpha);
        }
        out[j] = o;
        sv += o * o;
    }
    if (mode == 1) {
        __shared__ double red[4];
        const double s = block_sum(sv, red);
        if (threadIdx.x == 0) part[blockIdx.x] = s;
    }
}

// Build R (in place of N) and R⁻¹ for the current row scaling.  Throws if N is not SPD.
void dense_factor(System& S) {
    ensure_full_csr(S);   // AᵀA from GT
    hipStream_t st = S.stream;
    const int64_t n = S.G.n;
    const int64_t npad = (n + TB - 1) / TB * TB, ld = npad;
    const int nb = (int)(npad / TB);
    if (S.dR.n != npad * npad) {
        graph_cache_drop(&S);   // captured dense-preconditioned batches hold the old pointers
        S.dR.alloc(npad * npad);
        S.dRi.alloc(npad * npad);
    }
    S.dR.zero(st);
    S.dRi.zero(st);
    hipLaunchKernelGGL(k_normal_rows, dim3(grid_for(npad)), dim3(BLOCK), 0, st, n, npad, ld, S.GT.rp.p, S.GT.ci.p,
                       S.GT.val.p, S.G.rp.p, S.G.ci.p, S.G.val.p, S.rs.p, S.dR.p);
    KERNEL_CHECK();
    DBuf<int> err(1);
    err.zero(st);
    for (int kb = 0; kb < nb; ++kb) {
        const int64_t k0 = (int64_t)kb * TB;
        hipLaunchKernelGGL(k_potrf_diag, dim3(1), dim3(TW), 0, st, S.dR.p, ld, k0, err.p);
        const int m = nb - kb - 1;
        if (m > 0) {
            hipLaunchKernelGGL(k_trsm_panel, dim3(m), dim3(TW), 0, st, S.dR.p, ld, k0);
            hipLaunchKernelGGL(k_syrk_tiles, dim3(m * m), dim3(BLOCK), 0, st, S.dR.p, ld, k0, m);
        }
    }
    KERNEL_CHECK();
    hipLaunchKernelGGL(k_zero_lower, dim3(grid_for(npad * npad)), dim3(BLOCK), 0, st, S.dR.p, npad, ld);
    for (int ib = nb - 1; ib >= 0; --ib) {
        hipLaunchKernelGGL(k_trinv_diag, dim3(1), dim3(TW), 0, st, S.dR.p, S.dRi.p, ld, (int64_t)ib * TB);
        if (nb - 1 - ib > 0)
            hipLaunchKernelGGL(k_trinv_row, dim3(nb - 1 - ib), dim3(BLOCK), 0, st, S.dR.p, S.dRi.p, ld, ib);
    }
    KERNEL_CHECK();
    int h_err = 0;
    HIP_CHECK(hipMemcpyAsync(&h_err, err.p, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (h_err) throw std::invalid_argument("dense factor: AᵀA is not positive definite (rank-deficient system)");
    S.dense_ld = ld;
    S.dense_valid = true;
}

// In place: Nm (npad x npad, row-major, SPD on its upper triangle, identity on the padding) -> R
// (upper Cholesky factor), and Ri = R⁻¹.  err (device int) is set when a pivot is not positive.
// Asynchronous on `st` (multigrid coarsest level, mg.inc).
void dense_spd_factor(double* Nm, double* Ri, int64_t npad, int* err, hipStream_t st) {
    const int64_t ld = npad;
    const int nb = (int)(npad / TB);
    HIP_CHECK(hipMemsetAsync(Ri, 0, sizeof(double) * (size_t)(npad * npad), st));
    for (int kb = 0; kb < nb; ++kb) {
        const int64_t k0 = (int64_t)kb * TB;
        hipLaunchKernelGGL(k_potrf_diag, dim3(1), dim3(TW), 0, st, Nm, ld, k0, err);
        const int m = nb - kb - 1;
        if (m > 0) {
            hipLaunchKernelGGL(k_trsm_panel, dim3(m), dim3(TW), 0, st, Nm, ld, k0);
            hipLaunchKernelGGL(k_syrk_tiles, dim3(m * m), dim3(BLOCK), 0, st, Nm, ld, k0, m);
        }
    }
    hipLaunchKernelGGL(k_zero_lower, dim3(grid_for(npad * npad)), dim3(BLOCK), 0, st, Nm, npad, ld);
    for (int ib = nb - 1; ib >= 0; --ib) {
        hipLaunchKernelGGL(k_trinv_diag, dim3(1), dim3(TW), 0, st, Nm, Ri, ld, (int64_t)ib * TB);
        if (nb - 1 - ib > 0) hipLaunchKernelGGL(k_trinv_row, dim3(nb - 1 - ib), dim3(BLOCK), 0, st, Nm, Ri, ld, ib);
    }
    KERNEL_CHECK();
}

void dense_rowrss(System& S, double* dE) {
    const int64_t n = S.G.n;
    hipLaunchKernelGGL(k_rowrss_dense, dim3((unsigned)((n + 3) / 4)), dim3(BLOCK), 0, S.stream, S.dRi.p, n,
                       S.dense_ld, dE);
    KERNEL_CHECK();
}

}  // namespace lsq
