// rde.hip — order statistics of scaled residuals for smooth_fit's outlier editing (SURVEY.md §8(f)
// row 1; LSsurf/RDE.py:10-18, LSsurf/calc_sigma_extra.py:13-44).
//
// calc_sigma_extra searches σ_x with RDE(r / sqrt(σ_x² + σ²)) = 1, where RDE is half the 16–84
// percentile spread — a full sort per evaluation (25–30 evaluations per outer iteration, 2–8 M
// points).  Here r and σ stay on the device; an evaluation scales, radix-sorts and returns the
// requested order statistics, and the host does numpy's interpolation and scipy's bounded Brent
// search unchanged.  The scaling is evaluated exactly as numpy does (s·s + σ·σ, correctly
// rounded sqrt and divide, compiled with -ffp-contract=off), so the sorted values — and every
// editing decision — are bit-identical to the host path.
#include <hipcub/hipcub.hpp>

#include <string>

#include "../../include/lsqsurf.h"
#include "common.hpp"

struct lsq_rde {
    int device = 0;
    hipStream_t stream = nullptr;
    int64_t n = 0;
    lsq::DBuf<double> r, sig, x, xs;
    lsq::DBuf<unsigned char> tmp;
    size_t tmp_bytes = 0;
    std::string err;
};

namespace {

__global__ __launch_bounds__(lsq::BLOCK) void k_scaled(int64_t n, const double* __restrict__ r,
                                                       const double* __restrict__ sig, double s,
                                                       double* __restrict__ x) {
    const double s2 = s * s;
    for (int64_t i = (int64_t)blockIdx.x * lsq::BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * lsq::BLOCK) {
        const double q = sig[i] * sig[i];
        x[i] = r[i] / sqrt(s2 + q);
    }
}

__global__ void k_pick(int64_t n, const double* __restrict__ xs, int64_t m, const int64_t* __restrict__ idx,
                       double* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) out[k] = xs[idx[k]];
}

}  // namespace

extern "C" {

lsq_rde* lsq_rde_create(int32_t device, int64_t n, const double* r, const double* sigma) {
    if (n < 1 || !r || !sigma) return nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    auto* c = new lsq_rde();
    try {
        HIP_CHECK(hipSetDevice(device));
        c->device = device;
        HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->n = n;
        c->r.alloc(n);
        c->sig.alloc(n);
        c->x.alloc(n);
        c->xs.alloc(n);
        c->r.upload(r, n, c->stream);
        c->sig.upload(sigma, n, c->stream);
        HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, c->tmp_bytes, c->x.p, c->xs.p, (int)n, 0, 64,
                                                    c->stream));
        c->tmp.alloc((int64_t)c->tmp_bytes + 1);
        HIP_CHECK(hipStreamSynchronize(c->stream));
    } catch (const std::exception&) {
        lsq_rde_destroy(c);
        return nullptr;
    }
    return c;
}

int lsq_rde_order_stats(lsq_rde* c, double sigma_extra, int64_t n_idx, const int64_t* idx, double* out) {
    if (!c) return -1;
    try {
        if (n_idx < 0 || (n_idx && (!idx || !out))) throw std::invalid_argument("lsq_rde_order_stats: bad args");
        for (int64_t k = 0; k < n_idx; ++k)
            if (idx[k] < 0 || idx[k] >= c->n) throw std::invalid_argument("lsq_rde_order_stats: index out of range");
        HIP_CHECK(hipSetDevice(c->device));
        hipLaunchKernelGGL(k_scaled, dim3(lsq::grid_for(c->n)), dim3(lsq::BLOCK), 0, c->stream, c->n, c->r.p,
                           c->sig.p, sigma_extra, c->x.p);
        KERNEL_CHECK();
        HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(c->tmp.p, c->tmp_bytes, c->x.p, c->xs.p, (int)c->n, 0, 64,
                                                    c->stream));
        if (n_idx) {
            lsq::DBuf<int64_t> di(n_idx);
            lsq::DBuf<double> dout(n_idx);
            di.upload(idx, n_idx, c->stream);
            hipLaunchKernelGGL(k_pick, dim3((unsigned)((n_idx + 63) / 64)), dim3(64), 0, c->stream, c->n, c->xs.p, n_idx,
                               di.p, dout.p);
            KERNEL_CHECK();
            dout.download(out, n_idx, c->stream);
            HIP_CHECK(hipStreamSynchronize(c->stream));
        }
        return 0;
    } catch (const std::invalid_argument& e) {
        c->err = e.what();
        return -2;
    } catch (const std::exception& e) {
        c->err = e.what();
        return -3;
    }
}

const char* lsq_rde_last_error(lsq_rde* c) { return c ? c->err.c_str() : "null rde context"; }

void lsq_rde_destroy(lsq_rde* c) {
    if (!c) return;
    c->r.release();
    c->sig.release();
    c->x.release();
    c->xs.release();
    c->tmp.release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

}  // extern "C"
