// lsqr.hip — LSQR (Paige & Saunders 1982; scipy.sparse.linalg.lsqr's recurrences and stopping
// rules) on the device-resident SELL-64 system.  Replaces sparseqr.solve at
// LSsurf/smooth_fit.py:142.
//
// One iteration = four launches, all scalars stay on the device (no host round trip):
//   k_xw_spmv   [x/w update of the previous iteration  ‖  u ← (A ṽ)/α − α ũ/β ] + Σu², Σw²
//   k_beta      β = ‖u‖, ‖A‖ update                          (1 block, deterministic reduce)
//   k_spmtv     ṽ' ← (Aᵀ ũ)/β − β ṽ/α                         + Σṽ'²
//   k_givens    α = ‖ṽ'‖, plane rotation, norms, stopping test (1 block)
// ũ and ṽ are kept UNNORMALISED; the 1/β and 1/α scalings are folded into the next product,
// so normalisation costs no extra pass over HBM.  ṽ ping-pongs between two buffers.  Batches
// of iterations are captured once into a hipGraph and replayed; the host reads the 200-byte
// state only between batches.  Right preconditioning by column scaling is baked into the SELL
// values (A·D), and x = D y is applied on the way out.
#include <array>
#include <chrono>
#include <memory>
#include <stdexcept>
#include <cmath>
#include <vector>

#include "system.hpp"
#include "../../include/lsqsurf.h"

namespace lsq {

namespace {

constexpr int NPART = 2048;   // partial-sum slots per reduction (fixed grid => deterministic)

// ---- SELL-64 row kernel body: one lane = one row, 4 entries in flight per step -------------
__device__ __forceinline__ double sell_row_dot(const int32_t* __restrict__ ci, const double* __restrict__ val,
                                               int64_t base, int64_t W, int lane,
                                               const double* __restrict__ x) {
    const int32_t* c = ci + base + lane;
    const double* v = val + base + lane;
    double a0 = 0.0, a1 = 0.0;
    int64_t k = 0;
    for (; k + 4 <= W; k += 4) {
        const int32_t c0 = c[(k + 0) * SELL_C], c1 = c[(k + 1) * SELL_C];
        const int32_t c2 = c[(k + 2) * SELL_C], c3 = c[(k + 3) * SELL_C];
        const double v0 = v[(k + 0) * SELL_C], v1 = v[(k + 1) * SELL_C];
        const double v2 = v[(k + 2) * SELL_C], v3 = v[(k + 3) * SELL_C];
        a0 += v0 * x[c0];
        a1 += v1 * x[c1];
        a0 += v2 * x[c2];
        a1 += v3 * x[c3];
    }
    for (; k < W; ++k) a0 += v[k * SELL_C] * x[c[k * SELL_C]];
    return a0 + a1;
}

// partial-sum epilogue: one value per block into part[blockIdx-relative slot]
__device__ __forceinline__ void store_partial(double acc, double* part, int slot) {
    __shared__ double red[4];
    const double s = block_sum(acc, red);
    if (threadIdx.x == 0) part[slot] = s;
}

// ---- init: u = rs∘b − A y0 ; partials Σu², Σ(rs∘b)² -----------------------------------------
__global__ __launch_bounds__(BLOCK) void k_init_u(int64_t m, int64_t nslices, const int64_t* __restrict__ sp,
                                                  const int32_t* __restrict__ ci, const double* __restrict__ val,
                                                  const double* __restrict__ rs, const double* __restrict__ b,
                                                  const double* __restrict__ y0, const int32_t* __restrict__ perm,
                                                  double* __restrict__ u, double* __restrict__ bw, double* part_u,
                                                  double* part_b) {
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
    double su = 0.0, sb = 0.0;
    for (int64_t s = (int64_t)blockIdx.x * 4 + wid; s < nslices; s += (int64_t)gridDim.x * 4) {
        const int64_t row = s * SELL_C + lane;
        double ax = 0.0;
        if (y0 && row < m) {
            const int64_t base = sp[s];
            ax = sell_row_dot(ci, val, base, (sp[s + 1] - base) / SELL_C, lane, y0);
        }
        if (row < m) {
            const int64_t q = perm[row];   // u lives in A's SELL row order; b, rs in CSR order
            const double bb = rs[q] * b[q];
            const double uu = bb - ax;
            bw[row] = bb;
            u[row] = uu;
            su += uu * uu;
            sb += bb * bb;
        }
    }
    store_partial(su, part_u, blockIdx.x);
    store_partial(sb, part_b, blockIdx.x);
}

// ---- merged: x/w update (blocks [0,gX)) ‖ SpMV u-update (blocks [gX, gX+gA)) ----------------
__global__ __launch_bounds__(BLOCK) void k_xw_spmv(const LsqState* __restrict__ st, int gX,
                                                   int64_t n, double* __restrict__ y, double* __restrict__ w,
                                                   const double* __restrict__ vt, const double* __restrict__ xs,
                                                   int xs_scaled, int64_t m, int64_t nslices,
                                                   const int64_t* __restrict__ sp, const int32_t* __restrict__ ci,
                                                   const double* __restrict__ val, double* __restrict__ u,
                                                   double* part_u, double* part_w) {
    if ((int)blockIdx.x < gX) {
        // x/w update for the iteration whose rotation k_givens just finished
        if (st->finished || !st->have_xw) return;
        const double t1 = st->t1, t2 = st->t2, ia = st->inv_alpha;
        double sw = 0.0;
        for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gX * BLOCK) {
            const double wj = w[j];
            y[j] += t1 * wj;
            const double wn = vt[j] * ia + t2 * wj;
            w[j] = wn;
            sw += wn * wn;
        }
        store_partial(sw, part_w, blockIdx.x);
        return;
    }
    if (st->stop) return;
    const int bid = blockIdx.x - gX, gA = gridDim.x - gX;
    const double alpha = st->alpha, ib = st->inv_beta;
    const double ia = xs_scaled ? st->inv_alpha : 1.0;   // precond 2 gathers z = R⁻¹ ṽ/α
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
    double su = 0.0;
    for (int64_t s = (int64_t)bid * 4 + wid; s < nslices; s += (int64_t)gA * 4) {
        const int64_t row = s * SELL_C + lane;
        if (row < m) {
            const int64_t base = sp[s];
            const double ax = sell_row_dot(ci, val, base, (sp[s + 1] - base) / SELL_C, lane, xs);
            const double un = ax * ia - alpha * (u[row] * ib);
            u[row] = un;
            su += un * un;
        }
    }
    store_partial(su, part_u, bid);
}

// ---- SpMTV: ṽ' = (Aᵀ ũ)/β − β ṽ/α ; Σṽ'² --------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_spmtv(const LsqState* __restrict__ st, int64_t n, int64_t nslices,
                                                 const int64_t* __restrict__ sp, const int32_t* __restrict__ ci,
                                                 const double* __restrict__ val, const double* __restrict__ u,
                                                 const double* __restrict__ vin, double* __restrict__ vout,
                                                 double* part_v, int raw) {
    if (st->stop) return;
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
    const double ib = st->inv_beta, beta = st->beta, ia = st->inv_alpha;
    const bool skip = st->skip_v;
    double sv = 0.0;
    for (int64_t s = (int64_t)blockIdx.x * 4 + wid; s < nslices; s += (int64_t)gridDim.x * 4) {
        const int64_t row = s * SELL_C + lane;
        double vn;
        if (skip && !raw) {
            vn = row < n ? vin[row] : 0.0;
        } else if (row < n) {
            const int64_t base = sp[s];
            const double atu = sell_row_dot(ci, val, base, (sp[s + 1] - base) / SELL_C, lane, u);
            vn = raw ? atu : atu * ib - beta * (vin[row] * ia);   // raw: t = Aᵀũ for the R⁻ᵀ epilogue
        } else {
            vn = 0.0;
        }
        if (row < n) {
            vout[row] = vn;
            sv += vn * vn;
        }
    }
    store_partial(sv, part_v, blockIdx.x);
}

// deterministic single-block sum of nparts partials
__device__ double reduce_parts(const double* part, int nparts) {
    __shared__ double red[4];
    double a = 0.0;   // same summation order as a plain strided loop, 8 loads in flight
    for (int i0 = threadIdx.x; i0 < nparts; i0 += 8 * BLOCK) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = i0 + u * BLOCK < nparts ? part[i0 + u * BLOCK] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u) a += v[u];
    }
    return block_sum(a, red);  // valid in thread 0
}

// ---- β: 1-block kernel --------------------------------------------------------------------------
// mode 0: iteration; mode 1: init (also bnorm from part_b)
__global__ __launch_bounds__(BLOCK) void k_beta(LsqState* st, const double* part_u, int nu,
                                                const double* part_b, int nb, int mode, const double* gs) {
    if (mode == 0 && st->stop) {
        if (threadIdx.x == 0) st->finished = 1;   // the final x/w update has been applied
        return;
    }
    // gs: sums already reduced (and all-reduced across ranks): gs[0] = Σu², gs[3] = Σb²
    const double su = gs ? gs[0] : reduce_parts(part_u, nu);
    double sb = 0.0;
    if (mode == 1) sb = gs ? gs[3] : reduce_parts(part_b, nb);
    if (threadIdx.x) return;
    const double beta = sqrt(su);
    st->beta = beta;
    st->skip_v = !(beta > 0.0);
    if (beta > 0.0) st->inv_beta = 1.0 / beta;
    if (mode == 1) {
        st->bnorm = sqrt(sb);
        st->alpha = 0.0;
        st->inv_alpha = 0.0;
    } else if (beta > 0.0) {
        const double a = st->alpha;
        st->anorm = sqrt(st->anorm * st->anorm + a * a + beta * beta);
    }
}

__device__ __forceinline__ double sgn(double x) { return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : 0.0); }

// scipy _sym_ortho: stable Givens (c, s, r) with r = sqrt(a²+b²)
__device__ void sym_ortho(double a, double b, double& c, double& s, double& r) {
    if (b == 0.0) { c = sgn(a); s = 0.0; r = fabs(a); return; }
    if (a == 0.0) { c = 0.0; s = sgn(b); r = fabs(b); return; }
    if (fabs(b) > fabs(a)) {
        const double tau = a / b;
        s = sgn(b) / sqrt(1.0 + tau * tau);
        c = s * tau;
        r = b / s;
    } else {
        const double tau = b / a;
        c = sgn(a) / sqrt(1.0 + tau * tau);
        s = c * tau;
        r = a / c;
    }
}

// ---- α, rotation, norm estimates, stopping rules: 1-block kernel ----------------------------
// mode 1: init (rhobar = α, φ̄ = β ...); mode 0: iteration
__global__ __launch_bounds__(BLOCK) void k_givens(LsqState* st, const double* part_v, int nv,
                                                  const double* part_w, int nw, int mode, const double* gs) {
    if (mode == 0 && st->stop) return;
    // gs: gs[1] = Σw², gs[2] = Σṽ² (reduced across ranks)
    const double sv = gs ? gs[2] : reduce_parts(part_v, nv);
    const double sw = gs ? gs[1] : reduce_parts(part_w, nw);
    if (threadIdx.x) return;
    const double eps = 2.220446049250313e-16;
    if (!st->skip_v) {
        const double alpha = sqrt(sv);
        st->alpha = alpha;
        st->inv_alpha = alpha > 0.0 ? 1.0 / alpha : 0.0;
    }
    const double alpha = st->alpha, beta = st->beta;
    if (mode == 1) {
        st->rhobar = alpha;
        st->phibar = beta;
        st->rnorm = beta;
        st->r1norm = beta;
        st->r2norm = beta;
        st->arnorm = alpha * beta;
        st->itn = 0;
        st->have_xw = 0;
        st->finished = 0;
        st->stop = 0;
        st->istop = 0;
        if (alpha * beta == 0.0) {   // exact solution x = x0
            st->stop = 1;
            st->finished = 1;
        }
        return;
    }
    // ddnorm uses w before this iteration's update: ‖w_k‖² = sw (from the previous x/w pass)
    st->itn += 1;
    double cs, sn, rho;
    sym_ortho(st->rhobar, beta, cs, sn, rho);
    const double theta = sn * alpha;
    st->rhobar = -cs * alpha;
    const double phi = cs * st->phibar;
    st->phibar = sn * st->phibar;
    const double tau = sn * phi;
    st->t1 = phi / rho;
    st->t2 = -theta / rho;
    st->ddnorm += sw / (rho * rho);
    const double delta = st->sn2 * rho;
    const double gambar = -st->cs2 * rho;
    const double rhs = phi - delta * st->z;
    const double zbar = rhs / gambar;
    st->xnorm = sqrt(st->xxnorm + zbar * zbar);
    const double gamma = sqrt(gambar * gambar + theta * theta);
    st->cs2 = gambar / gamma;
    st->sn2 = theta / gamma;
    st->z = rhs / gamma;
    st->xxnorm += st->z * st->z;
    st->acond = st->anorm * sqrt(st->ddnorm);
    const double res1 = st->phibar * st->phibar;
    const double rnorm = sqrt(res1 + st->res2);
    st->rnorm = rnorm;
    st->arnorm = alpha * fabs(tau);
    st->r1norm = rnorm;
    st->r2norm = rnorm;
    st->have_xw = 1;
    const double bnorm = st->bnorm, anorm = st->anorm, xnorm = st->xnorm;
    const double test1 = rnorm / bnorm;
    const double test2 = st->arnorm / (anorm * rnorm + eps);
    const double test3 = 1.0 / (st->acond + eps);
    const double t1 = test1 / (1.0 + anorm * xnorm / bnorm);
    const double rtol = st->btol + st->atol * anorm * xnorm / bnorm;
    int istop = 0;
    if (st->itn >= st->maxit) istop = 7;
    if (!st->no_stop) {
        if (1.0 + test3 <= 1.0) istop = 6;
        if (1.0 + test2 <= 1.0) istop = 5;
        if (1.0 + t1 <= 1.0) istop = 4;
        if (test3 <= st->ctol) istop = 3;
        if (test2 <= st->atol) istop = 2;
        if (test1 <= rtol) istop = 1;
    }
    st->istop = istop;
    if (istop) st->stop = 1;
}

// w = ṽ/α, y = y0 (or 0), Σw²
__global__ __launch_bounds__(BLOCK) void k_init_w(const LsqState* __restrict__ st, int64_t n,
                                                  const double* __restrict__ vt, const double* __restrict__ y0s,
                                                  double* __restrict__ w, double* __restrict__ y, double* part_w) {
    const double ia = st->inv_alpha;
    double sw = 0.0;
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK) {
        const double wj = vt[j] * ia;
        w[j] = wj;
        y[j] = y0s ? y0s[j] : 0.0;
        sw += wj * wj;
    }
    store_partial(sw, part_w, blockIdx.x);
}

// y0s = x0 / cs  (warm start into preconditioned coordinates);  x = cs ∘ y on the way out
__global__ __launch_bounds__(BLOCK) void k_scale(int64_t n, const double* __restrict__ a, const double* __restrict__ cs,
                                                 int divide, double* __restrict__ out) {
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK)
        out[j] = divide ? a[j] / cs[j] : a[j] * cs[j];
}

// ---- distributed helpers ---------------------------------------------------------------------
// gs[slot_a] = Σ part_a, gs[slot_b] = Σ part_b (rank-local, deterministic), before the all-reduce
__global__ __launch_bounds__(BLOCK) void k_red_parts(const double* part_a, int na, int slot_a, const double* part_b,
                                                     int nb, int slot_b, double* gs) {
    const double a = reduce_parts(part_a, na);
    double b = 0.0;
    if (part_b) b = reduce_parts(part_b, nb);
    if (threadIdx.x == 0) {
        gs[slot_a] = a;
        if (part_b) gs[slot_b] = b;
    }
}

// ṽ'_j = t_j/β − β ṽ_j/α over owned columns (after the reverse halo), Σṽ'²
__global__ __launch_bounds__(BLOCK) void k_vepi(const LsqState* __restrict__ st, int64_t n,
                                                const double* __restrict__ t, const double* __restrict__ vin,
                                                double* __restrict__ vout, double* part_v) {
    if (st->stop) return;
    const double ib = st->inv_beta, beta = st->beta, ia = st->inv_alpha;
    const bool skip = st->skip_v;
    double sv = 0.0;
    for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLOCK) {
        const double vn = skip ? vin[j] : t[j] * ib - beta * (vin[j] * ia);
        vout[j] = vn;
        sv += vn * vn;
    }
    store_partial(sv, part_v, blockIdx.x);
}

__global__ __launch_bounds__(BLOCK) void k_pack(int64_t cnt, const int32_t* __restrict__ idx,
                                                const double* __restrict__ src, double* __restrict__ dst) {
    for (int64_t k = (int64_t)blockIdx.x * BLOCK + threadIdx.x; k < cnt; k += (int64_t)gridDim.x * BLOCK)
        dst[k] = src[idx[k]];
}

// k_pack + k_red_parts in one launch (distributed CG): block 0 first reduces the step's scalar
// partials into gs (k_red_parts' summation order), then every block packs
__global__ __launch_bounds__(BLOCK) void k_pack_red(int64_t cnt, const int32_t* __restrict__ idx,
                                                    const double* __restrict__ src, double* __restrict__ dst,
                                                    const double* part_a, int na, int slot_a, const double* part_b,
                                                    int nb, int slot_b, double* gs) {
    if (blockIdx.x == 0) {
        const double a = reduce_parts(part_a, na);
        double b = 0.0;
        if (part_b) b = reduce_parts(part_b, nb);
        if (threadIdx.x == 0) {
            gs[slot_a] = a;
            if (part_b) gs[slot_b] = b;
        }
    }
    for (int64_t k = (int64_t)blockIdx.x * BLOCK + threadIdx.x; k < cnt; k += (int64_t)gridDim.x * BLOCK)
        dst[k] = src[idx[k]];
}

__global__ __launch_bounds__(BLOCK) void k_scatter_add(int64_t cnt, const int32_t* __restrict__ idx,
                                                       const double* __restrict__ src, double* __restrict__ dst) {
    for (int64_t k = (int64_t)blockIdx.x * BLOCK + threadIdx.x; k < cnt; k += (int64_t)gridDim.x * BLOCK)
        dst[idx[k]] += src[k];
}

#include "lsqr_mf.inc"
#include "lsqr_block.inc"

struct Grids {
    int gA, gT, gX, gR, gRT, gE;
    int gD, gS, gM, gXf;   // stencil operator: data-row blocks, node blocks, Aᵀu blocks, x/w blocks
    int gB;                // block-Jacobi epilogue
    size_t lds;            // dynamic LDS of k_mf_fwd (staged zv bands)
};

Grids grids_for(const System& S) {
    Grids g;
    g.gD = g.gS = g.gM = g.gXf = 1;
    // block-Jacobi epilogue: at most 1 024 workgroups (two thirds of one dispatch round at its 6 waves
    // per SIMD; 2 048 took 1.3 rounds): LSQR at C4 846–848 → 860–862 it/s (profiles/r06_lsqr_epi_ab.txt)
    g.gB = grid_for(std::max<int64_t>(S.nblk, 1) * 16, BLOCK, 1024);   // 16 lanes per column block
    g.lds = 0;
    if (S.mf)
        for (int k = 0; k < S.mfh.n_grids; ++k) g.lds = std::max<size_t>(g.lds, sizeof(double) * S.mfh.g[k].lds);

    if (S.mf) {
        g.gD = (int)std::min<int64_t>(std::max<int64_t>((S.Ad.nslices + 3) / 4, 1), NPART / 4);
        g.gS = (int)std::min<int64_t>(std::max<int64_t>(S.mfh.nodes / MF_ALIGN, 1), NPART - g.gD);
        g.gM = (int)std::min<int64_t>(std::max<int64_t>(S.mfh.nodes / (SELL_C * MF_NPT) / 4, 1), NPART);
        g.gXf = grid_for(S.n_full, BLOCK * 4, NPART);
    }
    g.gA = (int)std::min<int64_t>(std::max<int64_t>((S.A.nslices + 3) / 4, 1), NPART);
    g.gT = (int)std::min<int64_t>(std::max<int64_t>((S.AT.nslices + 3) / 4, 1), NPART);
    g.gX = grid_for(S.ncols_own(), BLOCK * 4, NPART);
    g.gR = grid_for(S.G.n, 4, NPART);        // k_gemv_upper: one wave per row
    g.gRT = grid_for(S.G.n, BLOCK, NPART);   // k_gemvT_upper: one thread per column
    g.gE = grid_for(S.ncols_own(), BLOCK * 4, NPART);
    return g;
}

void ensure_workspace(System& S) {
    const int64_t m = S.G.m, n = std::max<int64_t>(S.vlen(), 1);
    if (S.u.n != std::max<int64_t>(m, 1)) {
        S.u.alloc(std::max<int64_t>(m, 1));
        S.bw.alloc(std::max<int64_t>(m, 1));
    }
    if (S.vb0.n != n) {
        S.vb0.alloc(n);
        S.vb1.alloc(n);
        S.w.alloc(n);
        S.y.alloc(n);
        S.zt.alloc(n);
        S.tt.alloc(n);
    }
    if (!S.part_u.p) {
        S.part_u.alloc(NPART);
        S.part_v.alloc(NPART);
        S.part_w.alloc(NPART);
        S.part_b.alloc(NPART);
        S.st.alloc(1);
    }
}

// launch one LSQR iteration; parity p: ṽ read from vb[p], written to vb[1-p]
void launch_iteration(System& S, const Grids& g, int p, int precond) {
    hipStream_t st = S.stream;
    double* vt = p ? S.vb1.p : S.vb0.p;
    double* vo = p ? S.vb0.p : S.vb1.p;
    const bool dense = precond == 2, block = precond == 3, band = precond == 5;
    if (dense)   // z = R⁻¹ ṽ / α
        hipLaunchKernelGGL(k_gemv_upper, dim3(g.gR), dim3(BLOCK), 0, st, S.dRi.p, S.G.n, S.dense_ld, vt, S.st.p, 1,
                           S.zt.p);
    if (band)    // z = M ṽ / α, M = P S R̃⁻¹ (band back substitution)
        band_launch_bsub(S, vt, 1, S.zt.p);
    // gathered vector: ṽ (values carry cs), R⁻¹ṽ/α (dense / band), or z = M ṽ from the block epilogue
    hipLaunchKernelGGL(k_xw_spmv, dim3(g.gX + g.gA), dim3(BLOCK), 0, st, S.st.p, g.gX, S.G.n, S.y.p, S.w.p, vt,
                       (dense || block || band) ? S.zt.p : vt, (dense || band) ? 0 : 1, S.G.m, S.A.nslices, S.A.sp.p,
                       S.A.ci.p, S.A.val.p, S.u.p, S.part_u.p, S.part_w.p);
    hipLaunchKernelGGL(k_beta, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_u.p, g.gA, S.part_b.p, 0, 0, nullptr);
    if (block) {
        hipLaunchKernelGGL(k_spmtv, dim3(g.gT), dim3(BLOCK), 0, st, S.st.p, S.G.n, S.AT.nslices, S.AT.sp.p, S.AT.ci.p,
                           S.AT.val.p, S.u.p, vt, S.tt.p, S.part_v.p, 1);
        launch_block_epi(S, false, g.gB, S.tt.p, vt, vo, S.zt.p);
        hipLaunchKernelGGL(k_givens, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_v.p, g.gB, S.part_w.p, g.gX, 0, nullptr);
    } else if (dense) {
        hipLaunchKernelGGL(k_spmtv, dim3(g.gT), dim3(BLOCK), 0, st, S.st.p, S.G.n, S.AT.nslices, S.AT.sp.p, S.AT.ci.p,
                           S.AT.val.p, S.u.p, vt, S.tt.p, S.part_v.p, 1);
        hipLaunchKernelGGL(k_gemvT_upper, dim3(g.gRT), dim3(BLOCK), 0, st, S.dRi.p, S.G.n, S.dense_ld, S.tt.p, S.st.p,
                           1, vt, vo, S.part_v.p);
        hipLaunchKernelGGL(k_givens, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_v.p, g.gRT, S.part_w.p, g.gX, 0, nullptr);
    } else if (band) {   // raw Aᵀũ, then ṽ' = Mᵀ t/β − βṽ/α by the band forward substitution
        hipLaunchKernelGGL(k_spmtv, dim3(g.gT), dim3(BLOCK), 0, st, S.st.p, S.G.n, S.AT.nslices, S.AT.sp.p, S.AT.ci.p,
                           S.AT.val.p, S.u.p, vt, S.tt.p, S.part_v.p, 1);
        band_launch_fsub(S, S.tt.p, vt, vo, S.part_v.p);
        hipLaunchKernelGGL(k_givens, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_v.p, 1, S.part_w.p, g.gX, 0, nullptr);
    } else {
        hipLaunchKernelGGL(k_spmtv, dim3(g.gT), dim3(BLOCK), 0, st, S.st.p, S.G.n, S.AT.nslices, S.AT.sp.p, S.AT.ci.p,
                           S.AT.val.p, S.u.p, vt, vo, S.part_v.p, 0);
        hipLaunchKernelGGL(k_givens, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_v.p, g.gT, S.part_w.p, g.gX, 0, nullptr);
    }
}

// one iteration on the structured stencil operator (full column space, zv = cs∘ṽ)
void launch_iteration_mf(System& S, const Grids& g, int p, int precond) {
    hipStream_t st = S.stream;
    double* vt = p ? S.vb1.p : S.vb0.p;
    double* vo = p ? S.vb0.p : S.vb1.p;
    hipLaunchKernelGGL(k_mf_fwd_for(S), dim3(g.gXf + g.gD + g.gS), dim3(BLOCK), g.lds, st, S.st.p, g.gXf, g.gD, S.n_full, S.y.p,
                       S.w.p, vt, S.mfh.npts, S.Ad.nslices, S.Ad.sp.p, S.Ad.ci.p, S.Ad.val.p, S.mfd.p, S.zv.p, S.rs.p,
                       S.u.p, S.part_u.p, S.part_w.p);
    hipLaunchKernelGGL(k_beta, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_u.p, g.gD + g.gS, S.part_b.p, 0, 0,
                       nullptr);
    if (precond == 3) {   // raw Aᵀũ, then ṽ' = M^T t/β − βṽ/α and zv = M ṽ' per column block
        hipLaunchKernelGGL(k_mf_spmtv_for(S), dim3(g.gM), dim3(BLOCK), 0, st, S.st.p, S.ATd.rp.p, S.ATd.ci.p, S.ATd.val.p,
                           S.mfd.p, S.u.p, S.rs.p, S.csf.p, vt, S.tt.p, S.zv.p, S.part_v.p, 1);
        launch_block_epi(S, true, g.gB, S.tt.p, vt, vo, S.zv.p);
        hipLaunchKernelGGL(k_givens, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_v.p, g.gB, S.part_w.p, g.gXf, 0,
                           nullptr);
        return;
    }
    hipLaunchKernelGGL(k_mf_spmtv_for(S), dim3(g.gM), dim3(BLOCK), 0, st, S.st.p, S.ATd.rp.p, S.ATd.ci.p, S.ATd.val.p,
                       S.mfd.p, S.u.p, S.rs.p, S.csf.p, vt, vo, S.zv.p, S.part_v.p, 0);
    hipLaunchKernelGGL(k_givens, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_v.p, g.gM, S.part_w.p, g.gXf, 0, nullptr);
}

// final x/w update of a solve that stopped on the last iteration of a batch (newest ṽ in vb0)
void launch_flush(System& S, const Grids& g, bool mf) {
    if (mf) {
        hipLaunchKernelGGL(k_mf_fwd_for(S), dim3(g.gXf + g.gD + g.gS), dim3(BLOCK), g.lds, S.stream, S.st.p, g.gXf, g.gD,
                           S.n_full, S.y.p, S.w.p, S.vb0.p, S.mfh.npts, S.Ad.nslices, S.Ad.sp.p, S.Ad.ci.p, S.Ad.val.p,
                           S.mfd.p, S.zv.p, S.rs.p, S.u.p, S.part_u.p, S.part_w.p);
        hipLaunchKernelGGL(k_beta, dim3(1), dim3(BLOCK), 0, S.stream, S.st.p, S.part_u.p, g.gD + g.gS, S.part_b.p, 0, 0,
                           nullptr);
        KERNEL_CHECK();
        return;
    }
    hipLaunchKernelGGL(k_xw_spmv, dim3(g.gX + g.gA), dim3(BLOCK), 0, S.stream, S.st.p, g.gX, S.ncols_own(), S.y.p, S.w.p,
                       S.vb0.p, S.vb0.p, 1, S.G.m, S.A.nslices, S.A.sp.p, S.A.ci.p, S.A.val.p, S.u.p, S.part_u.p,
                       S.part_w.p);
    hipLaunchKernelGGL(k_beta, dim3(1), dim3(BLOCK), 0, S.stream, S.st.p, S.part_u.p, g.gA, S.part_b.p, 0, 0, nullptr);
    KERNEL_CHECK();
}

}  // namespace

// b on the device for a solve: rows [0, b_rows) from the host, the rest zero (lsq_opts.b_rows;
// C4's b is 75 M rows of which the 2 M data rows are non-zero: uploading it whole from pageable
// memory was most of the per-solve set-up), into the persistent S.rhs
const double* upload_rhs(System& S, const double* h_b, const lsq_opts& o, hipStream_t st) {
    const int64_t m = S.G.m, nb = o.b_rows > 0 && o.b_rows < m ? o.b_rows : m;
    if (S.rhs.n < std::max<int64_t>(m, 1)) S.rhs.alloc(std::max<int64_t>(m, 1));
    S.rhs.upload(h_b, nb, st);
    if (nb < m) HIP_CHECK(hipMemsetAsync(S.rhs.p + nb, 0, (size_t)(m - nb) * sizeof(double), st));
    return S.rhs.p;
}

// Initialise the LSQR state from rhs b (host, length m, unweighted) and optional warm start
// x0 (host, length n, or nullptr).  Mirrors scipy lsqr's set-up block for the operator A·M
// (M = diag(cs) for precond 0/1, M = R⁻¹ for precond 2).
namespace {

// lsqr_init on the structured stencil operator (full column space)
void lsqr_init_mf(System& S, const double* h_b, const double* h_x0, const lsq_opts& o, bool no_stop) {
    hipStream_t st = S.stream;
    ensure_workspace(S);
    const Grids g = grids_for(S);
    const int64_t n = S.G.n, nf = S.n_full;
    const double* dbp = upload_rhs(S, h_b, o, st);
    DBuf<double> dx0, dy0, dz0;
    if (h_x0) {
        dx0.alloc(std::max<int64_t>(n, 1));
        dx0.upload(h_x0, n, st);
        dy0.alloc(std::max<int64_t>(nf, 1));
        dz0.alloc(std::max<int64_t>(nf, 1));
        dy0.zero(st);
        dz0.zero(st);
        if (o.precond == 3)   // y0 = M⁻¹ x0 per block, z0 = x0 (full space)
            hipLaunchKernelGGL(k_block_warm, dim3(grid_for(S.nblk)), dim3(BLOCK), 0, st, S.nblk, S.blk_kmax * (S.blk_kmax + 1) / 2, S.blk_ptr.p,
                               S.blk_cols.p, S.blk_full.p, S.blk_Ri.p, dx0.p, dy0.p, dz0.p);
        else
            hipLaunchKernelGGL(k_mf_warm, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, S.keep.p, dx0.p, S.cs.p, dy0.p,
                               dz0.p);
        KERNEL_CHECK();
    }
    LsqState h{};
    h.atol = o.atol;
    h.btol = o.btol;
    h.ctol = o.conlim > 0 ? 1.0 / o.conlim : 0.0;
    h.maxit = o.maxit > 0 ? o.maxit : 4 * std::max<int64_t>(n, 1);
    h.no_stop = no_stop ? 1 : 0;
    h.cs2 = -1.0;
    HIP_CHECK(hipMemcpyAsync(S.st.p, &h, sizeof(h), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_mf_init_u_for(S), dim3(g.gD + g.gS), dim3(BLOCK), 0, st, g.gD, S.mfh.npts, S.Ad.nslices, S.Ad.sp.p,
                       S.Ad.ci.p, S.Ad.val.p, S.Ad.perm.p, S.mfd.p, h_x0 ? dz0.p : nullptr, S.rs.p, dbp, S.u.p, S.bw.p,
                       S.part_u.p, S.part_b.p);
    KERNEL_CHECK();
    hipLaunchKernelGGL(k_beta, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_u.p, g.gD + g.gS, S.part_b.p,
                       g.gD + g.gS, 1, nullptr);
    S.vb1.zero(st);
    if (o.precond == 3) {
        S.vb0.zero(st);   // columns outside every block (removed by Ip_c) stay 0
        S.zv.zero(st);
        hipLaunchKernelGGL(k_mf_spmtv_for(S), dim3(g.gM), dim3(BLOCK), 0, st, S.st.p, S.ATd.rp.p, S.ATd.ci.p, S.ATd.val.p,
                           S.mfd.p, S.u.p, S.rs.p, S.csf.p, S.vb1.p, S.tt.p, S.zv.p, S.part_v.p, 1);
        launch_block_epi(S, true, g.gB, S.tt.p, S.vb1.p, S.vb0.p, S.zv.p);
        hipLaunchKernelGGL(k_givens, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_v.p, g.gB, S.part_w.p, g.gXf, 1,
                           nullptr);
    } else {
        hipLaunchKernelGGL(k_mf_spmtv_for(S), dim3(g.gM), dim3(BLOCK), 0, st, S.st.p, S.ATd.rp.p, S.ATd.ci.p, S.ATd.val.p,
                           S.mfd.p, S.u.p, S.rs.p, S.csf.p, S.vb1.p, S.vb0.p, S.zv.p, S.part_v.p, 0);
        hipLaunchKernelGGL(k_givens, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_v.p, g.gM, S.part_w.p, g.gXf, 1,
                           nullptr);
    }
    hipLaunchKernelGGL(k_init_w, dim3(g.gXf), dim3(BLOCK), 0, st, S.st.p, nf, S.vb0.p, h_x0 ? dy0.p : nullptr, S.w.p,
                       S.y.p, S.part_w.p);
    KERNEL_CHECK();
    HIP_CHECK(hipStreamSynchronize(st));
    S.iter_parity = 0;
}

}  // namespace

void lsqr_init(System& S, const double* h_b, const double* h_x0, const lsq_opts& o, bool no_stop, bool mf) {
    if (mf) return lsqr_init_mf(S, h_b, h_x0, o, no_stop);
    hipStream_t st = S.stream;
    ensure_workspace(S);
    const Grids g = grids_for(S);
    const int64_t m = S.G.m, n = S.G.n;
    const bool dense = o.precond == 2, block = o.precond == 3, band = o.precond == 5;
    const double* dbp = upload_rhs(S, h_b, o, st);
    DBuf<double> dx0, dy0;
    if (h_x0) {
        dx0.alloc(std::max<int64_t>(n, 1));
        dy0.alloc(std::max<int64_t>(n, 1));
        dx0.upload(h_x0, n, st);
        if (block) {   // y0 = M⁻¹ x0 per block; the SELL values are unscaled, so A·M·y0 = A x0
            hipLaunchKernelGGL(k_block_warm, dim3(grid_for(S.nblk)), dim3(BLOCK), 0, st, S.nblk, S.blk_kmax * (S.blk_kmax + 1) / 2, S.blk_ptr.p,
                               S.blk_cols.p, S.blk_cols.p, S.blk_Ri.p, dx0.p, dy0.p, S.zt.p);
        } else if (dense) {   // y0 = R x0 ; the SELL values are unscaled, so A·M·y0 = A x0
            hipLaunchKernelGGL(k_gemv_upper, dim3(g.gR), dim3(BLOCK), 0, st, S.dR.p, n, S.dense_ld, dx0.p, nullptr, 2,
                               dy0.p);
        } else if (band) {    // y0 = M⁻¹ x0 = R̃ S⁻¹ Pᵀ x0
            band_launch_warm(S, dx0.p, dy0.p);
        } else {       // y0 = x0 / cs ; A·D·y0 = A x0 with the scaled SELL values
            hipLaunchKernelGGL(k_scale, dim3(grid_for(n)), dim3(BLOCK), 0, st, n, dx0.p, S.cs.p, 1, dy0.p);
        }
        KERNEL_CHECK();
    }
    LsqState h{};
    h.atol = o.atol;
    h.btol = o.btol;
    h.ctol = o.conlim > 0 ? 1.0 / o.conlim : 0.0;
    h.maxit = o.maxit > 0 ? o.maxit : 4 * std::max<int64_t>(n, 1);
    h.no_stop = no_stop ? 1 : 0;
    h.cs2 = -1.0;
    HIP_CHECK(hipMemcpyAsync(S.st.p, &h, sizeof(h), hipMemcpyHostToDevice, st));
    // the SpMV of the warm start gathers in A·M coordinates: y0 for precond 0/1, x0 for 2 and 3
    const double* gather0 = h_x0 ? ((dense || block || band) ? dx0.p : dy0.p) : nullptr;
    hipLaunchKernelGGL(k_init_u, dim3(g.gA), dim3(BLOCK), 0, st, m, S.A.nslices, S.A.sp.p, S.A.ci.p, S.A.val.p,
                       S.rs.p, dbp, gather0, S.A.perm.p, S.u.p, S.bw.p, S.part_u.p, S.part_b.p);
    KERNEL_CHECK();
    hipLaunchKernelGGL(k_beta, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_u.p, g.gA, S.part_b.p, g.gA, 1, nullptr);
    KERNEL_CHECK();
    S.vb1.zero(st);
    int nv = g.gT;
    if (block) {
        hipLaunchKernelGGL(k_spmtv, dim3(g.gT), dim3(BLOCK), 0, st, S.st.p, n, S.AT.nslices, S.AT.sp.p, S.AT.ci.p,
                           S.AT.val.p, S.u.p, S.vb1.p, S.tt.p, S.part_v.p, 1);
        launch_block_epi(S, false, g.gB, S.tt.p, S.vb1.p, S.vb0.p, S.zt.p);
        nv = g.gB;
    } else if (dense) {
        hipLaunchKernelGGL(k_spmtv, dim3(g.gT), dim3(BLOCK), 0, st, S.st.p, n, S.AT.nslices, S.AT.sp.p, S.AT.ci.p,
                           S.AT.val.p, S.u.p, S.vb1.p, S.tt.p, S.part_v.p, 1);
        hipLaunchKernelGGL(k_gemvT_upper, dim3(g.gRT), dim3(BLOCK), 0, st, S.dRi.p, n, S.dense_ld, S.tt.p, S.st.p, 1,
                           S.vb1.p, S.vb0.p, S.part_v.p);
        nv = g.gRT;
    } else if (band) {
        hipLaunchKernelGGL(k_spmtv, dim3(g.gT), dim3(BLOCK), 0, st, S.st.p, n, S.AT.nslices, S.AT.sp.p, S.AT.ci.p,
                           S.AT.val.p, S.u.p, S.vb1.p, S.tt.p, S.part_v.p, 1);
        band_launch_fsub(S, S.tt.p, S.vb1.p, S.vb0.p, S.part_v.p);
        nv = 1;
    } else {
        hipLaunchKernelGGL(k_spmtv, dim3(g.gT), dim3(BLOCK), 0, st, S.st.p, n, S.AT.nslices, S.AT.sp.p, S.AT.ci.p,
                           S.AT.val.p, S.u.p, S.vb1.p, S.vb0.p, S.part_v.p, 0);
    }
    KERNEL_CHECK();
    hipLaunchKernelGGL(k_givens, dim3(1), dim3(BLOCK), 0, st, S.st.p, S.part_v.p, nv, S.part_w.p, g.gX, 1, nullptr);
    KERNEL_CHECK();
    hipLaunchKernelGGL(k_init_w, dim3(g.gX), dim3(BLOCK), 0, st, S.st.p, n, S.vb0.p, h_x0 ? dy0.p : nullptr, S.w.p,
                       S.y.p, S.part_w.p);
    KERNEL_CHECK();
    HIP_CHECK(hipStreamSynchronize(st));   // db / dx0 / dy0 are released on return
    S.iter_parity = 0;
}

namespace {

struct GraphCache {
    const System* sys = nullptr;
    const void* key = nullptr;   // S.u.p identifies the workspace generation
    int batch = 0;
    int mode = -1;               // precond * 2 + stencil-operator flag
    hipGraphExec_t exec = nullptr;
};
thread_local GraphCache g_cache;
thread_local GraphCache g_cache_cg;   // CGNR iteration batches (lsqr_cg.inc)
thread_local GraphCache g_cache_group;   // a one-rank RCCL group's CGNR batches (lsqr_cg_dist.inc)

void launch_any(System& S, const Grids& g, int p, int precond, bool mf) {
    if (mf)
        launch_iteration_mf(S, g, p, precond);
    else
        launch_iteration(S, g, p, precond);
}

// run `count` iterations starting at parity S.iter_parity (count even when graphs are used)
void run_batch(System& S, int count, bool use_graph, int precond, bool mf) {
    const Grids g = grids_for(S);
    const int mode = precond * 2 + (mf ? 1 : 0);
    if (use_graph && count % 2 == 0 && S.iter_parity == 0) {
        GraphCache& c = g_cache;
        if (c.exec == nullptr || c.sys != &S || c.key != (const void*)S.u.p || c.batch != count || c.mode != mode) {
            if (c.exec) (void)hipGraphExecDestroy(c.exec);
            c.exec = nullptr;
            hipGraph_t graph;
            HIP_CHECK(hipStreamBeginCapture(S.stream, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < count; ++i) launch_any(S, g, i & 1, precond, mf);
            HIP_CHECK(hipStreamEndCapture(S.stream, &graph));
            HIP_CHECK(hipGraphInstantiate(&c.exec, graph, nullptr, nullptr, 0));
            HIP_CHECK(hipGraphDestroy(graph));
            c.sys = &S;
            c.key = S.u.p;
            c.batch = count;
            c.mode = mode;
        }
        HIP_CHECK(hipGraphLaunch(c.exec, S.stream));
        return;
    }
    for (int i = 0; i < count; ++i) {
        launch_any(S, g, S.iter_parity, precond, mf);
        S.iter_parity ^= 1;
    }
    KERNEL_CHECK();
}

// Algorithmic HBM bytes per launch of the two streaming kernels (DESIGN.md §Byte model).
// Assembled SELL: x/w+A·v = 12Z + 16m + 48n, Aᵀu = 12Z + 8m + 16n (Z = nnz, 12 B per entry).
// Stencil operator (n_f full columns, Z_d entries of the m_d data rows, stencil part p with
// n_p rows): x/w+A·v = 48 n_f + 12 Z_d + 16 m_d + Σ_p n_p (16 + 8 [row scale not constant] +
// 8 nfield [field-valued]); Aᵀu = 36 n_f + 12 Z_d + 8 m_d + Σ_p n_p (8 + 8 [...] + 8 nfield [...]).
// Per column: y, w read+write, ṽ, zv
// gathered once / cs, ṽ in, ṽ out, zv out, the 4-B ATd row offset.
void kernel_bytes(const System& S, bool mf, double out[2]) {
    if (mf) {
        const double nf = (double)S.n_full, md = (double)S.mfh.npts, zd = (double)S.GdT.nnz;
        double f = 48.0 * nf + 12.0 * zd + 16.0 * md, t = 36.0 * nf + 12.0 * zd + 8.0 * md;
        for (int p = 0; p < S.mfh.n_parts; ++p) {
            const double n = (double)S.mfh.p[p].n_eq, w = S.mfh.p[p].wconst ? 0.0 : 8.0;
            const double fv = S.mfh.p[p].var ? 8.0 * S.mfh.p[p].nfield : 0.0;   // per-row field values
            f += n * (16.0 + w + fv);
            t += n * (8.0 + w + fv);
        }
        out[0] = f;
        out[1] = t;
        return;
    }
    const double Z = (double)S.G.nnz, m = (double)S.G.m, n = (double)S.G.n;
    out[0] = 12.0 * Z + 16.0 * m + 48.0 * n;
    out[1] = 12.0 * Z + 8.0 * m + 16.0 * n;
}

}  // namespace

// Jacobi column scale of the structured system: squared norms in the full space (scratch: csf),
// then cs_j = 1/‖A_j‖ (or the squared norm, raw) for the compact columns.
void mf_column_scale(System& S, bool raw) {
    hipLaunchKernelGGL(k_mf_colnorm, dim3(grid_for(S.mfh.nodes)), dim3(BLOCK), 0, S.stream, S.mfd.p, S.ATd.perm.p,
                       S.GdT.rp.p, S.GdT.ci.p, S.GdT.val.p, S.rs.p, S.csf.p);
    KERNEL_CHECK();
    hipLaunchKernelGGL(k_norm_gather, dim3(grid_for(S.G.n)), dim3(BLOCK), 0, S.stream, S.G.n, S.keep.p, S.csf.p,
                       raw ? 1 : 0, S.cs.p);
    KERNEL_CHECK();
}

// Bytes per LSQR iteration with preconditioner `precond`.  Block-Jacobi (3): Aᵀu writes the raw
// t = Aᵀũ (8 B per column instead of cs, ṽ in, ṽ out and zv: 24 B less per column of the
// structured v-space, 8 B less on the assembled one) and the epilogue k_block_epi(_aff) reads t,
// ṽ, writes ṽ', z (32 B per block column) and streams the factor: the lf_t copy (sizeof(lf_t)·npks
// per block, k_block_epi_lf) or the f64 one (8·npk).
double bytes_per_iter(const System& S, bool mf, int precond) {
    double b[2];
    kernel_bytes(S, mf, b);
    double tot = b[0] + b[1];
    if (precond == 3 && S.nblk > 0) {
        const int npk = S.blk_kmax * (S.blk_kmax + 1) / 2;
        const double ncol = S.blk_affine ? (double)S.nblk * S.blk_kmax : (double)S.G.n;
        const double fac = block_epi_lf(S, mf) ? (double)sizeof(lf_t) * lf_stride(npk) : 8.0 * npk;
        tot -= mf ? 24.0 * (double)S.n_full : 8.0 * (double)S.G.n;
        tot += 32.0 * ncol + fac * (double)S.nblk;
    }
    return tot;
}

namespace {

void fill_stats(const LsqState& h, lsq_stats* s) {
    s->iters = h.itn;
    s->istop = h.istop;
    s->r1norm = h.r1norm;
    s->r2norm = h.r2norm;
    s->anorm = h.anorm;
    s->acond = h.acond;
    s->arnorm = h.arnorm;
    s->xnorm = h.xnorm;
}

bool use_mf(const System& S, const lsq_opts& o) {
    return S.mf && o.op == 0 && o.precond != 2 && o.precond != 5 && !S.dist;
}

void prepare(System& S, int precond, bool mf) {
    if (!mf) ensure_sell(S);
    refresh_scaling(S, precond);
    if (precond == 2 && !S.dense_valid) dense_factor(S);
    if (precond == 3 && !S.blk_valid) block_factor(S);
    if (precond == 5 && !S.band.valid) band_precond(S);
}

}  // namespace

void graph_cache_drop(const System* S) {
    for (GraphCache* c : {&g_cache, &g_cache_cg, &g_cache_group})
        if (c->sys == S && c->exec) {
            (void)hipGraphExecDestroy(c->exec);
            *c = GraphCache{};
        }
    if (S && S->mg) mg_graph_drop(S->mg);
}

int lsqr_solve(System& S, const double* h_b, double* h_x, const lsq_opts& o, lsq_stats* stats) {
    const bool mf = use_mf(S, o);
    prepare(S, o.precond, mf);
    lsqr_init(S, h_b, o.use_x0 ? h_x : nullptr, o, false, mf);
    int batch = o.batch > 0 ? o.batch : 16;
    batch += batch & 1;
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    HIP_CHECK(hipEventRecord(e0, S.stream));
    LsqState h{};
    HIP_CHECK(hipMemcpyAsync(&h, S.st.p, sizeof(h), hipMemcpyDeviceToHost, S.stream));
    HIP_CHECK(hipStreamSynchronize(S.stream));
    while (!h.stop) {
        run_batch(S, batch, o.use_graph != 0, o.precond, mf);
        HIP_CHECK(hipMemcpyAsync(&h, S.st.p, sizeof(h), hipMemcpyDeviceToHost, S.stream));
        HIP_CHECK(hipStreamSynchronize(S.stream));
    }
    const Grids g = grids_for(S);
    if (!h.finished) {   // stop on the last iteration of a batch: apply its x/w update
        S.iter_parity = 0;
        launch_flush(S, g, mf);
    }
    HIP_CHECK(hipEventRecord(e1, S.stream));
    const int64_t n = S.G.n;
    if (o.precond == 3)   // x = M y, block by block, into compact positions
        hipLaunchKernelGGL(k_block_x, dim3(grid_for(S.nblk)), dim3(BLOCK), 0, S.stream, S.nblk,
                           S.blk_kmax * (S.blk_kmax + 1) / 2, S.blk_ptr.p,
                           S.blk_cols.p, mf ? S.blk_full.p : S.blk_cols.p, S.blk_Ri.p, S.y.p, S.vb1.p);
    else if (mf)
        hipLaunchKernelGGL(k_mf_x, dim3(grid_for(n)), dim3(BLOCK), 0, S.stream, n, S.keep.p, S.y.p, S.csf.p, S.vb1.p);
    else if (o.precond == 2)
        hipLaunchKernelGGL(k_gemv_upper, dim3(g.gR), dim3(BLOCK), 0, S.stream, S.dRi.p, n, S.dense_ld, S.y.p, nullptr,
                           2, S.vb1.p);
    else if (o.precond == 5)
        band_launch_bsub(S, S.y.p, 2, S.vb1.p);
    else
        hipLaunchKernelGGL(k_scale, dim3(grid_for(n)), dim3(BLOCK), 0, S.stream, n, S.y.p, S.cs.p, 0, S.vb1.p);
    KERNEL_CHECK();
    S.vb1.download(h_x, n, S.stream);
    HIP_CHECK(hipMemcpyAsync(&h, S.st.p, sizeof(h), hipMemcpyDeviceToHost, S.stream));
    HIP_CHECK(hipStreamSynchronize(S.stream));
    if (o.precond == 5) band_check(S);
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (stats) {
        fill_stats(h, stats);
        stats->time_s = ms * 1e-3;
        stats->bytes_per_iter = bytes_per_iter(S, mf, o.precond);
    }
    S.iter_ready = false;   // the solve consumed the iteration state
    return h.istop == 7 ? 1 : 0;
}

int lsqr_iterate(System& S, const double* h_b, int64_t iters, const lsq_opts& o, lsq_stats* stats) {
    const bool mf = use_mf(S, o);
    const int mode = o.precond * 2 + (mf ? 1 : 0);
    prepare(S, o.precond, mf);
    if (!S.iter_ready || S.iter_mode != mode) {
        lsq_opts oo = o;
        oo.maxit = INT64_MAX / 4;
        lsqr_init(S, h_b, nullptr, oo, true, mf);
        S.iter_ready = true;
        S.iter_mode = mode;
    }
    int batch = o.batch > 0 ? o.batch : 16;
    batch += batch & 1;
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    HIP_CHECK(hipEventRecord(e0, S.stream));
    int64_t left = iters;
    while (left > 0) {
        const int c = (int)std::min<int64_t>(left, batch);
        run_batch(S, c, o.use_graph != 0 && c == batch, o.precond, mf);
        left -= c;
    }
    HIP_CHECK(hipEventRecord(e1, S.stream));
    LsqState h{};
    HIP_CHECK(hipMemcpyAsync(&h, S.st.p, sizeof(h), hipMemcpyDeviceToHost, S.stream));
    HIP_CHECK(hipStreamSynchronize(S.stream));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (stats) {
        fill_stats(h, stats);
        stats->time_s = ms * 1e-3;
        stats->bytes_per_iter = bytes_per_iter(S, mf, o.precond);
    }
    return 0;
}

// Time each iteration kernel of operator `op` in isolation (reps launches, HIP events on the
// handle's stream) + algorithmic bytes per launch.  Destroys the iteration state; used by
// bench.py for the per-kernel roofline.
void lsqr_profile(System& S, int reps, int op, double* out /* [8] */) {
    lsq_opts o;
    lsq_default_opts(&o);
    o.op = op;
    const bool mf = S.dist ? S.dist_mf : use_mf(S, o);
    if (!S.dist) prepare(S, 1, mf);   // a distributed rank keeps the scaling its group filled
    ensure_workspace(S);
    const Grids g = grids_for(S);
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    LsqState h{};
    h.alpha = 1.0; h.inv_alpha = 1.0; h.beta = 1.0; h.inv_beta = 1.0; h.have_xw = 1; h.t1 = 1e-3; h.t2 = -1e-3;
    h.maxit = INT64_MAX / 4; h.no_stop = 1; h.bnorm = 1.0; h.cs2 = -1.0;
    HIP_CHECK(hipMemcpyAsync(S.st.p, &h, sizeof(h), hipMemcpyHostToDevice, S.stream));
    S.vb0.zero(S.stream);
    S.vb1.zero(S.stream);
    S.u.zero(S.stream);
    S.w.zero(S.stream);
    S.y.zero(S.stream);
    if (mf) S.zv.zero(S.stream);
    const int nu = mf ? g.gD + g.gS : g.gA, nv = mf ? g.gM : g.gT, nx = mf ? g.gXf : g.gX;
    for (int k = 0; k < 4; ++k) {
        for (int pass = 0; pass < 2; ++pass) {   // pass 0 = warm-up
            HIP_CHECK(hipEventRecord(e0, S.stream));
            for (int r = 0; r < reps; ++r) {
                if (k == 0 && mf)
                    hipLaunchKernelGGL(k_mf_fwd_for(S), dim3(g.gXf + g.gD + g.gS), dim3(BLOCK), g.lds, S.stream, S.st.p, g.gXf,
                                       g.gD, S.n_full, S.y.p, S.w.p, S.vb0.p, S.mfh.npts, S.Ad.nslices, S.Ad.sp.p,
                                       S.Ad.ci.p, S.Ad.val.p, S.mfd.p, S.zv.p, S.rs.p, S.u.p, S.part_u.p, S.part_w.p);
                else if (k == 0)
                    hipLaunchKernelGGL(k_xw_spmv, dim3(g.gX + g.gA), dim3(BLOCK), 0, S.stream, S.st.p, g.gX, S.G.n,
                                       S.y.p, S.w.p, S.vb0.p, S.vb0.p, 1, S.G.m, S.A.nslices, S.A.sp.p, S.A.ci.p,
                                       S.A.val.p, S.u.p, S.part_u.p, S.part_w.p);
                else if (k == 1 && mf)
                    hipLaunchKernelGGL(k_mf_spmtv_for(S), dim3(g.gM), dim3(BLOCK), 0, S.stream, S.st.p, S.ATd.rp.p,
                                       S.ATd.ci.p, S.ATd.val.p, S.mfd.p, S.u.p, S.rs.p, S.csf.p, S.vb0.p, S.vb1.p,
                                       S.zv.p, S.part_v.p, 0);
                else if (k == 1)
                    hipLaunchKernelGGL(k_spmtv, dim3(g.gT), dim3(BLOCK), 0, S.stream, S.st.p, S.G.n, S.AT.nslices,
                                       S.AT.sp.p, S.AT.ci.p, S.AT.val.p, S.u.p, S.vb0.p, S.vb1.p, S.part_v.p, 0);
                else if (k == 2)
                    hipLaunchKernelGGL(k_beta, dim3(1), dim3(BLOCK), 0, S.stream, S.st.p, S.part_u.p, nu,
                                       S.part_b.p, 0, 2, nullptr);
                else
                    hipLaunchKernelGGL(k_givens, dim3(1), dim3(BLOCK), 0, S.stream, S.st.p, S.part_v.p, nv,
                                       S.part_w.p, nx, 2, nullptr);
            }
            HIP_CHECK(hipEventRecord(e1, S.stream));
            HIP_CHECK(hipEventSynchronize(e1));
        }
        float ms = 0.f;
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        out[k] = ms / reps;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    kernel_bytes(S, mf, out + 4);
    out[6] = out[7] = 0.0;
    S.iter_ready = false;
}

// sqrt(diag((AᵀA)⁻¹)) for the current row weights / mask, via the dense factor.
void lsqr_sigma_x(System& S, double* h_E) {
    refresh_scaling(S, S.cs_mode < 0 ? 0 : S.cs_mode);
    if (!S.dense_valid) dense_factor(S);
    DBuf<double> dE(std::max<int64_t>(S.G.n, 1));
    dense_rowrss(S, dE.p);
    dE.download(h_E, S.G.n, S.stream);
    HIP_CHECK(hipStreamSynchronize(S.stream));
}

// Download R⁻¹ (n x n, row-major, upper triangular) of the dense factor.
void lsqr_get_rinv(System& S, double* h_Ri) {
    refresh_scaling(S, S.cs_mode < 0 ? 0 : S.cs_mode);
    if (!S.dense_valid) dense_factor(S);
    const int64_t n = S.G.n, ld = S.dense_ld;
    HIP_CHECK(hipMemcpy2DAsync(h_Ri, n * sizeof(double), S.dRi.p, ld * sizeof(double), n * sizeof(double), n,
                               hipMemcpyDeviceToHost, S.stream));
    HIP_CHECK(hipStreamSynchronize(S.stream));
}

#include "lsqr_cg.inc"

#include "lsqr_dist.inc"

#include "lsqr_cg_dist.inc"

}  // namespace lsq
