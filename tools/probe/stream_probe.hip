// Development probe: the HBM rate of the update kernel's access mix on this box, without its
// arithmetic.  n = C4's 12.58 M columns; per column the update reads q, s (16 B) and 13.3 B of
// factor and writes s, z (16 B).  Variants: plain double loads, 64 lanes per wave over contiguous
// columns (ideal), and 60 of 64 lanes (the update's 5 blocks × 12 lanes per wave).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int LANES, bool FACT, bool NT>
__global__ __launch_bounds__(256) void k_mix(int64_t n, const double* __restrict__ q, double* __restrict__ s,
                                             double* __restrict__ z, const double* __restrict__ f, int64_t nf,
                                             double alpha, double* __restrict__ part) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t nw = (int64_t)gridDim.x * 4;
    double acc = 0.0;
    for (int64_t c0 = ((int64_t)blockIdx.x * 4 + w) * LANES; c0 < n; c0 += nw * LANES) {
        const int64_t c = c0 + lane;
        const bool on = lane < LANES && c < n;
        const double qj = on ? q[c] : 0.0, sj = on ? s[c] : 0.0;
        double fv = 0.0;
        if (FACT) {   // 13.3 B per column: 5 words per 3 columns of factor, coalesced
            const int64_t fw0 = c0 * 5 / 3 / 4;   // in double2 units... approximate stream position
            const double2* f2 = reinterpret_cast<const double2*>(f);
            if (lane < (LANES * 5 / 6) && fw0 + lane < nf) { const double2 v = f2[fw0 + lane]; fv = v.x + v.y; }
        }
        const double sn = sj - alpha * qj, zn = sn * 0.5 + fv * 1e-300;
        if (on) {
            if (NT) { __builtin_nontemporal_store(sn, s + c); __builtin_nontemporal_store(zn, z + c); }
            else { s[c] = sn; z[c] = zn; }
        }
        acc += sn * zn;
    }
    if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

int main() {
    const int64_t n = 12582912, nf = n * 40 / 3 / 16;   // double2 words of a 13.3-B-per-column stream
    double *q, *s, *z, *f, *part;
    CK(hipMalloc(&q, n * 8)); CK(hipMalloc(&s, n * 8)); CK(hipMalloc(&z, n * 8));
    CK(hipMalloc(&f, nf * 16)); CK(hipMalloc(&part, 1 << 20));
    CK(hipMemset(q, 0, n * 8)); CK(hipMemset(s, 0, n * 8)); CK(hipMemset(z, 0, n * 8)); CK(hipMemset(f, 0, nf * 16));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto run = [&](auto kern, const char* name, double bytes, int grid) {
        for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, n, q, s, z, f, nf, 1e-3, part);
        hipEventRecord(a);
        const int it = 50;
        for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, n, q, s, z, f, nf, 1e-3, part);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double t = ms / 1e3 / it;
        printf("%-34s grid %6d  %7.1f us  %6.2f TB/s\n", name, grid, t * 1e6, bytes / t / 1e12);
    };
    const double b4 = 32.0 * n, b5 = b4 + 16.0 * nf;
    for (int grid : {2048, 4096, 8192}) {
        run(k_mix<64, false, false>, "64 lanes, q s -> s z", b4, grid);
        run(k_mix<64, false, true>, "64 lanes, q s -> s z, NT", b4, grid);
        run(k_mix<60, false, false>, "60 lanes, q s -> s z", b4, grid);
        run(k_mix<64, true, false>, "64 lanes + factor stream", b5, grid);
        run(k_mix<60, true, true>, "60 lanes + factor stream, NT", b5, grid);
    }
    return 0;
}
