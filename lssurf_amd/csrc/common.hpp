// common.hpp — shared device/host helpers for liblsqsurf (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace lsq {

constexpr int WAVE = 64;          // CDNA wavefront width (hard-coded, cdna_hip_programming §1)
constexpr int BLOCK = 256;        // 4 waves per workgroup
constexpr int SELL_C = 64;        // SELL slice height = one wave, one row per lane
constexpr int MAX_GRID = 2048;    // 256 CUs x 8 resident 256-thread blocks (Guideline 11)

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
// A request the library declines for lack of resources (device memory, band width): status -5,
// so a caller may fall back to another method instead of failing (everything else is an error).
struct Refused : std::invalid_argument {
    using std::invalid_argument::invalid_argument;
};

#define HIP_CHECK(expr)                                                                     \
    do {                                                                                    \
        hipError_t e__ = (expr);                                                            \
        if (e__ != hipSuccess)                                                              \
            throw ::lsq::HipError(std::string(#expr) + ": " + hipGetErrorString(e__) +      \
                                  " (" __FILE__ ":" + std::to_string(__LINE__) + ")");      \
    } while (0)

#define KERNEL_CHECK() HIP_CHECK(hipGetLastError())

inline int grid_for(int64_t work, int per_block = BLOCK, int cap = MAX_GRID) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

// ---- device reductions (deterministic: fixed shuffle tree, fixed LDS tree) -----------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Sum over a 256-thread block; result valid in thread 0.
__device__ __forceinline__ double block_sum(double v, double* lds4) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) lds4[wid] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) r = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
    __syncthreads();
    return r;
}

// Device buffer with RAII.
template <class T>
struct DBuf {
    T* p = nullptr;
    int64_t n = 0;
    DBuf() = default;
    explicit DBuf(int64_t count) { alloc(count); }
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    DBuf(DBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DBuf& operator=(DBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
        return *this;
    }
    ~DBuf() { release(); }
    void alloc(int64_t count) {
        release();
        n = count;
        if (count > 0) HIP_CHECK(hipMalloc(&p, sizeof(T) * (size_t)count));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void upload(const T* h, int64_t count, hipStream_t s) {
        if (count) HIP_CHECK(hipMemcpyAsync(p, h, sizeof(T) * count, hipMemcpyHostToDevice, s));
    }
    void download(T* h, int64_t count, hipStream_t s) const {
        if (count) HIP_CHECK(hipMemcpyAsync(h, p, sizeof(T) * count, hipMemcpyDeviceToHost, s));
    }
    void zero(hipStream_t s) {
        if (n) HIP_CHECK(hipMemsetAsync(p, 0, sizeof(T) * n, s));
    }
    size_t bytes() const { return sizeof(T) * (size_t)n; }
};

// Exclusive scan of n int64 values in place, returns the total (synchronises the stream).
int64_t exclusive_scan_i64(int64_t* d, int64_t n, hipStream_t s);

}  // namespace lsq
