// scan.hip — deterministic three-phase exclusive scan of int64 (setup-time only).
#include "common.hpp"

namespace lsq {

namespace {
constexpr int SCAN_BLOCKS = 1024;

// Phase 1: per-block sums of a contiguous chunk.
__global__ __launch_bounds__(BLOCK) void k_chunk_sum(const int64_t* __restrict__ d, int64_t n,
                                                     int64_t chunk, int64_t* __restrict__ sums) {
    const int64_t b0 = (int64_t)blockIdx.x * chunk;
    const int64_t b1 = b0 + chunk < n ? b0 + chunk : n;
    int64_t acc = 0;
    for (int64_t i = b0 + threadIdx.x; i < b1; i += BLOCK) acc += d[i];
    __shared__ int64_t red[BLOCK];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = BLOCK / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = red[0];
}

// Phase 2: exclusive scan of the (<= SCAN_BLOCKS) block sums by one block; total at sums[nb].
__global__ __launch_bounds__(1024) void k_scan_sums(int64_t* __restrict__ sums, int nb) {
    __shared__ int64_t s[1024];
    const int t = threadIdx.x;
    s[t] = t < nb ? sums[t] : 0;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive
        int64_t v = t >= o ? s[t - o] : 0;
        __syncthreads();
        s[t] += v;
        __syncthreads();
    }
    if (t < nb) sums[t] = t ? s[t - 1] : 0;
    if (t == 0) sums[nb] = s[1023];
}

// Phase 3: each block scans its chunk serially in BLOCK-sized tiles with a carry.
__global__ __launch_bounds__(BLOCK) void k_chunk_scan(int64_t* __restrict__ d, int64_t n, int64_t chunk,
                                                      const int64_t* __restrict__ sums) {
    const int64_t b0 = (int64_t)blockIdx.x * chunk;
    const int64_t b1 = b0 + chunk < n ? b0 + chunk : n;
    __shared__ int64_t s[BLOCK];
    int64_t carry = sums[blockIdx.x];
    for (int64_t base = b0; base < b1; base += BLOCK) {
        const int64_t i = base + threadIdx.x;
        int64_t v = i < b1 ? d[i] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < BLOCK; o <<= 1) {
            int64_t t = (int)threadIdx.x >= o ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < b1) d[i] = carry + s[threadIdx.x] - v;
        carry += s[BLOCK - 1];
        __syncthreads();
    }
}
}  // namespace

int64_t exclusive_scan_i64(int64_t* d, int64_t n, hipStream_t s) {
    if (n <= 0) return 0;
    int64_t chunk = (n + SCAN_BLOCKS - 1) / SCAN_BLOCKS;
    if (chunk < BLOCK) chunk = BLOCK;
    const int nb = (int)((n + chunk - 1) / chunk);
    DBuf<int64_t> sums(nb + 1);
    hipLaunchKernelGGL(k_chunk_sum, dim3(nb), dim3(BLOCK), 0, s, d, n, chunk, sums.p);
    KERNEL_CHECK();
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, s, sums.p, nb);
    KERNEL_CHECK();
    hipLaunchKernelGGL(k_chunk_scan, dim3(nb), dim3(BLOCK), 0, s, d, n, chunk, sums.p);
    KERNEL_CHECK();
    int64_t total = 0;
    HIP_CHECK(hipMemcpyAsync(&total, sums.p + nb, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    return total;
}

}  // namespace lsq
