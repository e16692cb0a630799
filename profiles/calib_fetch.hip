// calib_fetch.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the LSQR kernels use (MI355X_MICROARCH.md §HBM: only 16 B/lane is calibrated there).
// Each kernel streams a known number of bytes from a 2 GiB buffer (well past the 256 MiB
// Infinity Cache); run under `rocprofv3 --pmc FETCH_SIZE` (and WRITE_SIZE) and divide.
//   k_rd4   : 4 B/lane coalesced loads  (SELL column indices)
//   k_rd8   : 8 B/lane coalesced loads  (SELL values, dense vectors)
//   k_rd16  : 16 B/lane coalesced loads (reference point of the guide)
//   k_wr8   : 8 B/lane coalesced stores
//   k_gat8  : 8 B/lane random gathers from a 100 MB vector (x[ci] pattern, L2/L3 resident)
// Build: hipcc -O3 --offload-arch=gfx950 profiles/calib_fetch.hip -o /tmp/calib_fetch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

template <typename T>
__global__ void k_rd(const T* __restrict__ a, size_t n, double* __restrict__ out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = a[i];
        s += (double)reinterpret_cast<const unsigned char*>(&v)[0];
    }
    if (s == -1.0) out[0] = s;   // keeps the loads; never true
}

__global__ void k_wr8(double* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = (double)i;
}

__global__ void k_gat8(const double* __restrict__ x, const int* __restrict__ idx, size_t n, double* __restrict__ out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += x[idx[i]];
    if (s == -1.0) out[0] = s;
}

int main() {
    const size_t bytes = size_t(2) << 30;
    char* buf;
    double* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 8));
    CK(hipMemset(buf, 1, bytes));
    const int grid = 4096, block = 256;
    hipLaunchKernelGGL(k_rd<unsigned int>, dim3(grid), dim3(block), 0, 0, (const unsigned int*)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_rd<double>, dim3(grid), dim3(block), 0, 0, (const double*)buf, bytes / 8, out);
    hipLaunchKernelGGL(k_rd<double2>, dim3(grid), dim3(block), 0, 0, (const double2*)buf, bytes / 16, out);
    hipLaunchKernelGGL(k_wr8, dim3(grid), dim3(block), 0, 0, (double*)buf, bytes / 8);
    // gathers: 100 MB x, 256 Mi random indices (1 GiB) -> algorithmic 1 GiB idx + 2 GiB of x values
    const size_t nx = 100u << 17, ng = size_t(256) << 20;
    double* x;
    int* idx;
    CK(hipMalloc(&x, nx * 8));
    CK(hipMalloc(&idx, ng * 4));
    int* h = (int*)std::malloc(ng * 4);
    unsigned long long s = 88172645463325252ull;
    for (size_t i = 0; i < ng; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        h[i] = (int)(s % nx);
    }
    CK(hipMemcpy(idx, h, ng * 4, hipMemcpyHostToDevice));
    CK(hipMemset(x, 0, nx * 8));
    hipLaunchKernelGGL(k_gat8, dim3(grid), dim3(block), 0, 0, x, idx, ng, out);
    CK(hipDeviceSynchronize());
    std::printf("bytes per streaming kernel: %zu (KB %zu); gather: idx %zu B, x %zu B of a %zu B vector\n", bytes,
                bytes >> 10, ng * 4, ng * 8, nx * 8);
    std::free(h);
    return 0;
}
