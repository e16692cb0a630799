// system.hpp — the device-resident least-squares system behind an lsq_handle.
//
// HBM layout (DESIGN.md §Data layout):
//   G   canonical CSR of the formed, UNWEIGHTED operator [G_data; Gc]·Ip_c  (rp int64, ci int32,
//       val f64; rows in input order, columns ascending, duplicates summed, zeros dropped)
//   GT  its transpose (CSR, rows = columns of G, entries in ascending row order)
//   A   SELL-64 copy of diag(rs)·G·diag(cs) — rs = row weight × row mask, cs = column
//       preconditioner — one slice = 64 consecutive rows = one wavefront, column-major inside
//       the slice so lane l reads entry k of its row at sp[s] + 64k + l (fully coalesced)
//   AT  SELL-64 copy of the transpose, same scaling
// The SELL copies are what the LSQR iteration streams; G/GT keep the unweighted values so
// row weights / masks / preconditioner changes only re-fill values (no re-formation).
#pragma once
#include <string>

#include "common.hpp"

namespace lsq {

struct Csr {
    int64_t m = 0, n = 0, nnz = 0;
    DBuf<int64_t> rp;   // m+1
    DBuf<int32_t> ci;   // nnz
    DBuf<double> val;   // nnz
};

struct Sell {
    int64_t rows = 0, nslices = 0, nent = 0;
    DBuf<int64_t> sp;   // nslices+1 entry offsets (multiples of 64)
    DBuf<int32_t> ci;   // nent
    DBuf<double> val;   // nent (padding: val 0, col = a valid column of the row)
};

// LSQR scalar state, device resident (one per handle).  Field meanings follow
// scipy.sparse.linalg.lsqr's locals.
struct LsqState {
    double alpha, beta, inv_alpha, inv_beta;
    double rhobar, phibar, anorm, acond, ddnorm, res2, xnorm, xxnorm, z, cs2, sn2;
    double bnorm, t1, t2, rnorm, r1norm, r2norm, arnorm;
    double atol, btol, ctol;
    int64_t itn, maxit;
    int32_t istop;      // scipy istop
    int32_t stop;       // set by the alpha/givens kernel when istop != 0
    int32_t finished;   // set after the final x/w update of a stopped solve
    int32_t have_xw;    // t1/t2 of a completed iteration are pending application
    int32_t skip_v;     // beta == 0 in the current iteration
    int32_t no_stop;    // lsq_iterate: only maxit stops
    int32_t pad[2];
};

struct System {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // column map (Ip_c)
    int64_t n_full = 0, n_keep = 0;
    bool have_colmap = false;
    DBuf<int32_t> colmap;   // n_full -> compact index or -1

    Csr G, GT;
    DBuf<double> roww;      // m row weights (1 if unset)
    DBuf<uint8_t> rowkeep;  // m (1 keep)
    DBuf<double> rs;        // m effective row scale = roww * keep
    DBuf<double> cs;        // n column scale (preconditioner)
    int cs_mode = -1;       // precond the SELL values were filled with (-1 = stale)
    bool rs_dirty = true;
    Sell A, AT;

    // dense factor (precond 2 / error propagation): R and R⁻¹, npad x npad row-major
    DBuf<double> dR, dRi;
    int64_t dense_ld = 0;
    bool dense_valid = false;

    // LSQR workspace
    DBuf<double> u, vb0, vb1, w, y, bw, zt, tt;
    DBuf<double> part_u, part_v, part_w, part_b;
    DBuf<LsqState> st;
    bool iter_ready = false;   // lsq_iterate state initialised
    int iter_parity = 0;

    ~System();
};

// build.hip
void form_from_coo(System& S, int64_t m, int64_t n_full, int64_t nnz, const int64_t* r,
                   const int64_t* c, const double* v);
void finish_formation(System& S);              // G set -> GT, SELL copies, default scaling
void refresh_scaling(System& S, int precond);   // rs/cs -> SELL values
void csr_spmv(System& S, int trans, const double* dx, double* dy);  // unweighted G / Gᵀ products

// dense.hip
void dense_factor(System& S);                     // R, R⁻¹ of diag(rs)·G (throws if not SPD)
void dense_rowrss(System& S, double* dE);         // sqrt(row sums of R⁻¹²) = sqrt(diag((AᵀA)⁻¹))
__global__ void k_gemv_upper(const double* M, int64_t n, int64_t ld, const double* v, const LsqState* st,
                             int scale_mode, double* z);
__global__ void k_gemvT_upper(const double* M, int64_t n, int64_t ld, const double* t, const LsqState* st, int mode,
                              const double* vin, double* out, double* part);

}  // namespace lsq
