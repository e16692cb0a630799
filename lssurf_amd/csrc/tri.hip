// tri.hip — GPU replacements for LSsurf's Cython triangular kernels:
//   inv_tr_upper         (LSsurf/inv_tr_upper.pyx:19-94, caller smooth_fit.py:240-248)
//   propagate_qz_errors  (LSsurf/propagate_qz_errors.pyx:15-69)
//   spsolve_tr_upper     (LSsurf/spsolve_tr_upper.pyx:11-54)
//
// R^-1 columns are independent, so a workgroup solves 256 columns at once: lane b owns column
// col_b and all lanes sweep the SAME row i (descending), so the row's (j, R_ij) entries are
// broadcast loads and the workspace X[j][b] reads are coalesced across lanes.  Each lane runs
// exactly the Cython recurrence for its column — same operands, same order, no FMA contraction
// (this file is compiled with -ffp-contract=off) — so every emitted value is bit-identical.
// Lanes whose column is below the current row idle (< 256 rows of waste per workgroup).
#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/lsqsurf.h"
#include "common.hpp"

namespace lsq {
namespace {

thread_local std::string t_err;

// Solve columns [c0, c0+C) of R X = I restricted to rows 0..c0+C-1; X is (c0+C) x C, row-major.
__global__ __launch_bounds__(BLOCK) void k_tri_inv_cols(int64_t c0, int64_t C, const int32_t* __restrict__ rp,
                                                        const int32_t* __restrict__ ci,
                                                        const double* __restrict__ dv, double* __restrict__ X) {
    const int64_t b = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    const int64_t col = c0 + b;
    const bool active = b < C;
    // highest column handled by this workgroup
    const int64_t top = std::min<int64_t>(c0 + (int64_t)(blockIdx.x + 1) * BLOCK, c0 + C) - 1;
    for (int64_t i = top; i >= 0; --i) {
        if (!active || i > col) continue;          // this lane's column has not started yet
        double x = (i == col) ? 1.0 : 0.0;
        const int32_t s = rp[i], e = rp[i + 1];
        for (int32_t k = s + 1; k < e; ++k) {
            const int32_t j = ci[k];
            if (j > col) break;                     // x_j = 0 for j > col (sorted indices)
            x -= dv[k] * X[(int64_t)j * C + b];
        }
        x /= dv[s];
        X[i * C + b] = x;
    }
}

// per-column emission count (i == col or |x| > tol)
__global__ __launch_bounds__(BLOCK) void k_tri_count(int64_t c0, int64_t C, const double* __restrict__ X, double tol,
                                                     int64_t* __restrict__ cnt) {
    const int64_t b = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (b >= C) return;
    const int64_t col = c0 + b;
    int64_t k = 0;
    for (int64_t i = col; i >= 0; --i) {
        const double x = X[i * C + b];
        if (i == col || fabs(x) > tol) ++k;
    }
    cnt[b] = k;
}

// write emissions of column col at global offset off[b] (only those < limit)
__global__ __launch_bounds__(BLOCK) void k_tri_emit(int64_t c0, int64_t C, const double* __restrict__ X, double tol,
                                                    const int64_t* __restrict__ off, int64_t limit,
                                                    int32_t* __restrict__ rr, int32_t* __restrict__ cc,
                                                    double* __restrict__ vv) {
    const int64_t b = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (b >= C) return;
    const int64_t col = c0 + b;
    int64_t o = off[b];
    for (int64_t i = col; i >= 0 && o < limit; --i) {
        const double x = X[i * C + b];
        if (i == col || fabs(x) > tol) {
            rr[o] = (int32_t)i;
            cc[o] = (int32_t)col;
            vv[o] = x;
            ++o;
        }
    }
}

// E_i += sum over the chunk's columns, in column-descending order (propagate_qz_errors order)
__global__ __launch_bounds__(BLOCK) void k_tri_rss(int64_t c0, int64_t C, const double* __restrict__ X,
                                                   double* __restrict__ E) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= c0 + C) return;
    double e = E[i];
    for (int64_t b = C - 1; b >= 0; --b) {
        if (c0 + b < i) break;
        const double x = X[i * C + b];
        e += x * x;
    }
    E[i] = e;
}

__global__ void k_sqrt(int64_t n, double* __restrict__ E) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) E[i] = sqrt(E[i]);
}

// spsolve_tr_upper: the recurrence is a serial chain; one lane walks it (bit-identical order)
__global__ void k_tri_solve_serial(int64_t N, const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                   const double* __restrict__ dv, double* __restrict__ x) {
    if (blockIdx.x || threadIdx.x) return;
    for (int64_t i = N - 1; i >= 0; --i) {
        const int32_t s = rp[i], e = rp[i + 1];
        double t = x[i];
        for (int32_t k = s + 1; k < e; ++k) t -= dv[k] * x[ci[k]];
        t /= dv[s];
        x[i] = t;
    }
}

struct DevR {
    DBuf<int32_t> rp, ci;
    DBuf<double> dv;
};

void upload_R(DevR& R, int64_t N, const int32_t* indptr, const int32_t* indices, const double* data, hipStream_t s) {
    if (N <= 0) throw std::invalid_argument("N must be positive");
    if (!indptr || !indices || !data) throw std::invalid_argument("null R arrays");
    const int64_t nnz = indptr[N];
    for (int64_t i = 0; i < N; ++i)
        if (indptr[i + 1] <= indptr[i]) throw std::invalid_argument("row " + std::to_string(i) + " of R is empty");
    R.rp.alloc(N + 1);
    R.ci.alloc(std::max<int64_t>(nnz, 1));
    R.dv.alloc(std::max<int64_t>(nnz, 1));
    R.rp.upload(indptr, N + 1, s);
    R.ci.upload(indices, nnz, s);
    R.dv.upload(data, nnz, s);
}

int64_t chunk_cols(int64_t N) {
    const int64_t budget = (int64_t)4 << 30;   // 4 GiB of workspace per chunk
    int64_t C = budget / (8 * std::max<int64_t>(N, 1));
    C = std::max<int64_t>(C / BLOCK * BLOCK, BLOCK);
    return std::min<int64_t>(C, N);
}

template <class F>
int tri_guard(int32_t device, F&& f) {
    t_err.clear();
    try {
        int ndev = 0;
        HIP_CHECK(hipGetDeviceCount(&ndev));
        if (device < 0 || device >= ndev) throw std::invalid_argument("bad device");
        HIP_CHECK(hipSetDevice(device));
        return f();
    } catch (const std::invalid_argument& e) {
        t_err = e.what();
        return -2;
    } catch (const std::exception& e) {
        t_err = e.what();
        return -3;
    }
}

}  // namespace
}  // namespace lsq

using namespace lsq;

extern "C" {

const char* tri_last_error(void) { return t_err.c_str(); }

int tri_upper_solve_csr(int32_t device, int64_t N, const int32_t* indptr, const int32_t* indices, const double* data,
                        const double* b, double* x) {
    return tri_guard(device, [&]() {
        hipStream_t s = nullptr;
        DevR R;
        upload_R(R, N, indptr, indices, data, s);
        DBuf<double> dx(N);
        dx.upload(b, N, s);
        hipLaunchKernelGGL(k_tri_solve_serial, dim3(1), dim3(64), 0, s, N, R.rp.p, R.ci.p, R.dv.p, dx.p);
        KERNEL_CHECK();
        dx.download(x, N, s);
        HIP_CHECK(hipStreamSynchronize(s));
        return 0;
    });
}

int tri_upper_inv_csr(int32_t device, int64_t N, const int32_t* indptr, const int32_t* indices, const double* data,
                      int64_t nnz_max, float tol, int32_t* rr, int32_t* cc, double* vv, int64_t* n_out) {
    return tri_guard(device, [&]() {
        if (nnz_max < 1) throw std::invalid_argument("nnz_max must be >= 1");
        hipStream_t s = nullptr;
        DevR R;
        upload_R(R, N, indptr, indices, data, s);
        const double dtol = (double)tol;             // C float promoted, as in the .pyx
        const int64_t limit = nnz_max - 1;           // emissions that fit before status=1
        const int64_t Cmax = chunk_cols(N);
        DBuf<double> X((N) * Cmax);
        DBuf<int64_t> cnt(Cmax + 1);
        DBuf<int32_t> drr(std::max<int64_t>(std::min<int64_t>(limit, N * N), 1));
        DBuf<int32_t> dcc(drr.n);
        DBuf<double> dvv(drr.n);
        int64_t done = 0;   // emissions written so far (global order: col descending)
        int status = 0;
        std::vector<int64_t> hc(Cmax + 1);
        for (int64_t c1 = N; c1 > 0 && !status;) {
            const int64_t C = std::min<int64_t>(Cmax, c1);
            const int64_t c0 = c1 - C;
            const int gb = (int)((C + BLOCK - 1) / BLOCK);
            hipLaunchKernelGGL(k_tri_inv_cols, dim3(gb), dim3(BLOCK), 0, s, c0, C, R.rp.p, R.ci.p, R.dv.p, X.p);
            KERNEL_CHECK();
            hipLaunchKernelGGL(k_tri_count, dim3(gb), dim3(BLOCK), 0, s, c0, C, X.p, dtol, cnt.p);
            KERNEL_CHECK();
            cnt.download(hc.data(), C, s);
            HIP_CHECK(hipStreamSynchronize(s));
            // offsets in column-descending order
            std::vector<int64_t> off(C);
            int64_t acc = done;
            for (int64_t b = C - 1; b >= 0; --b) {
                off[b] = acc;
                acc += hc[b];
            }
            if (acc > limit) status = 1;   // inv_tr_upper breaks at emission index nnz-1
            const int64_t lim = std::min<int64_t>(acc, limit);
            if (lim > (int64_t)drr.n) throw std::runtime_error("emission buffer too small");
            cnt.upload(off.data(), C, s);
            hipLaunchKernelGGL(k_tri_emit, dim3(gb), dim3(BLOCK), 0, s, c0, C, X.p, dtol, cnt.p, lim, drr.p, dcc.p,
                               dvv.p);
            KERNEL_CHECK();
            HIP_CHECK(hipStreamSynchronize(s));
            done = lim;
            c1 = c0;
        }
        drr.download(rr, done, s);
        dcc.download(cc, done, s);
        dvv.download(vv, done, s);
        HIP_CHECK(hipStreamSynchronize(s));
        if (status) {   // the .pyx returns out_*[0:nnz] with the unwritten last slot still zero
            rr[limit] = 0;
            cc[limit] = 0;
            vv[limit] = 0.0;
            done = nnz_max;
        }
        *n_out = done;
        return status;
    });
}

int tri_upper_rowrss_csr(int32_t device, int64_t N, const int32_t* indptr, const int32_t* indices, const double* data,
                         double* E) {
    return tri_guard(device, [&]() {
        hipStream_t s = nullptr;
        DevR R;
        upload_R(R, N, indptr, indices, data, s);
        const int64_t Cmax = chunk_cols(N);
        DBuf<double> X(N * Cmax), dE(N);
        dE.zero(s);
        for (int64_t c1 = N; c1 > 0;) {
            const int64_t C = std::min<int64_t>(Cmax, c1);
            const int64_t c0 = c1 - C;
            const int gb = (int)((C + BLOCK - 1) / BLOCK);
            hipLaunchKernelGGL(k_tri_inv_cols, dim3(gb), dim3(BLOCK), 0, s, c0, C, R.rp.p, R.ci.p, R.dv.p, X.p);
            KERNEL_CHECK();
            hipLaunchKernelGGL(k_tri_rss, dim3((unsigned)((c1 + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, c0, C, X.p,
                               dE.p);
            KERNEL_CHECK();
            c1 = c0;
        }
        hipLaunchKernelGGL(k_sqrt, dim3((unsigned)((N + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, N, dE.p);
        KERNEL_CHECK();
        dE.download(E, N, s);
        HIP_CHECK(hipStreamSynchronize(s));
        return 0;
    });
}

}  // extern "C"
