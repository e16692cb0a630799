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
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lsqsurf.h"
#include "common.hpp"

namespace lsq {

struct Csr {
    int64_t m = 0, n = 0, nnz = 0;
    DBuf<int64_t> rp;   // m+1
    DBuf<int32_t> ci;   // nnz
    DBuf<double> val;   // nnz
};

// CSR with int32 offsets whose rows are a permutation of another CSR's rows (perm: row -> source
// row, -1 = empty); one lane walks one row (ATd: data-row entries of one column)
struct Csr32 {
    int64_t rows = 0, nnz = 0;
    DBuf<int32_t> rp, ci, perm;
    DBuf<double> val;
};

struct Sell {
    int64_t rows = 0, nslices = 0, nent = 0;
    DBuf<int64_t> sp;   // nslices+1 entry offsets (multiples of 64)
    DBuf<int32_t> ci;   // nent
    DBuf<double> val;   // nent (padding: val 0, col = a valid column of the row)
    DBuf<int32_t> perm; // SELL row -> CSR row (A only; empty = identity).  See build_sell.
};

// Structured stencil operator (lsq_set_matrix_stencil systems): the constraint rows are never
// stored — a stencil part is (grid, centre box lo..hi, ≤8 template offsets/values) and row
// r = row0 + ravel_box(c − lo) of centre c has entries val_t at column col0 + ravel(c + off_t).
// A·v and Aᵀu walk the grid nodes (one thread per node, all parts of its grid); only the data
// rows (bi/trilinear interpolation, irregular) stay assembled, as SELL copies Ad / ATd.  The
// v-space of this operator is the FULL column space [0, n_full): columns removed by the column
// map (Ip_c) carry column scale 0, so they never enter the iteration (x_j stays 0), which is the
// same LSQR as on the compacted matrix.
constexpr int MF_MAX_PARTS = 32, MF_MAX_GRID_PARTS = 16, MF_MAX_GRIDS = 4;
constexpr int MF_MAXT = 16;                  // template entries per part (constant parts: ≤ 8 from
                                             // lsq_stencil_desc; field-valued parts: ≤ 16)
constexpr int MF_NPT = 2;                    // nodes per thread per block iteration
constexpr int MF_ALIGN = 256 * MF_NPT;       // node-enumeration alignment of every grid
constexpr int MF_R = 3;                      // |template offset| <= MF_R (8 edge classes per side)
constexpr int MF_LDS_MAX = 4096;             // doubles of LDS per block for the A·v staging (32 KB)
struct FastDiv {            // n / d for 0 <= n < 2^31: (n * mul) >> (32 + shift)
    uint64_t mul;
    uint32_t shift, d;
};
inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f{};
    f.d = d;
    uint32_t s = 0;
    while ((uint64_t(1) << s) < d) ++s;
    f.shift = s;
    f.mul = (uint64_t)(((unsigned __int128)1 << (32 + s)) + d - 1) / d;   // ceil(2^(32+s) / d)
    return f;
}
// Field-valued (variable-coefficient) parts — lsq_set_stencil_fields, e.g. the anisotropic
// notebook's directional operator whose rows are scaled by a direction field: entry t of the row
// of centre k (k = ravel_box(c − lo)) is val[t] · F[fsel[t]·n_eq + k] (val = ±1 there), with F
// the nfield exact per-row values on the device.
struct MfPart {
    int32_t grid, ntpl, row0, n_eq;          // rows [row0, row0 + n_eq) (global row ids < 2^31)
    int32_t lo[3], hi[3], bstride[3];
    int32_t ilo[3], ihi[3];                  // centres whose every template entry hits the box
    int32_t off[MF_MAXT][3];
    int32_t doff[MF_MAXT];                   // column offset of template entry t  (Σ off·stride)
    int32_t boff[MF_MAXT];                   // row offset of template entry t     (Σ off·bstride)
    uint64_t mlo8[3], mhi8[3];               // template validity masks by edge class (MF_R), ≤ 8 entries: byte a
    uint64_t mlo[3][2], mhi[3][2];           // the same for ≤ 16 entries (field-valued parts): 16 bits per class,
                                             // class a of dim e at bit 16·(a mod 4) of word a / 4 (mf_mask)
    int32_t loff[MF_MAXT];                   // A·v: LDS offset of template t (MfGrid bands)
    int32_t wconst, var;                     // 1: every row of the part has row scale w; 1: field-valued
    double w;
    double val[MF_MAXT];
    int32_t fsel[MF_MAXT];                   // field-valued parts: field of template t
    int32_t nfield, pad2;
    const double* F;                         // field-valued parts: nfield × n_eq (device)
};
struct MfGrid {
    int32_t ndim, nparts;
    int32_t shape[3], col0, nodes, node0;    // node0: first position in the MF_ALIGN-aligned enumeration
    FastDiv fd[3];
    int32_t part[MF_MAX_GRID_PARTS];
    // A·v stages the zv values a block iteration's MF_ALIGN nodes gather in LDS: one band per
    // distinct template y offset, covering the in-row offsets [emin, emax] of that offset
    int32_t nband, lds;                      // lds = doubles staged (0: gather from HBM)
    int32_t band_oy[2 * MF_R + 1], band_emin[2 * MF_R + 1], band_len[2 * MF_R + 1], band_start[2 * MF_R + 1];
};
struct MfDesc {
    int32_t n_grids, n_parts;
    int64_t nodes;                 // end of the node enumeration (grids with parts, MF_ALIGN-aligned)
    int64_t npts, m, n_full;
    MfGrid g[MF_MAX_GRIDS];
    MfPart p[MF_MAX_PARTS];
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

// Banded Cholesky factor of the equilibrated, permuted normal matrix (band.hip):
// S Pᵀ(AᵀA)P S = R̃ᵀR̃ with R̃ upper, stored as T tile rows × (w+1) 64×64 tiles (tile (I, J) at
// (I·(w+1) + J − I)·4096), D_K = R̃_KK⁻¹, sc = the diagonal of S (new order, npad), perm: new
// position -> compact column.
struct BandFactor {
    int64_t n = 0, T = 0;
    int w = 0;
    DBuf<double> R, D, sc;
    DBuf<int32_t> perm;
    DBuf<double> part;         // multi-workgroup triangular solves: partial sums (2 × NW × 64)
    DBuf<uint64_t> bar;        // and their grid barrier
    bool valid = false;
};

// CGNR normal operator (lsqr_cg.inc): AᵀA of the stencil rows of one grid is a constant-coefficient
// stencil whose coefficients depend only on each node's boundary class (position within K_e of
// either end of dim e, else interior).  Tiles of CG_TX nodes of dim 1 × ty rows of dim 0 × all of
// dim 2 are staged in LDS with their halo; lane = dim-1 position, so a wave's class is uniform
// except on tiles at a dim-1 edge.
constexpr int CG_TX = 64;
constexpr int CG_MAX_OFF = 128;             // Galerkin coarse grids (mg.inc): 5×5 (dy, dx) × 5 dt
constexpr int CG_MAXI = 16;                 // (row, dim-2) items per wave of one tile
// Column mode (every grid: dim 2 ≤ CG_MAXT nodes, |dt| ≤ 2): a thread owns a whole dim-2 column
// (y, x, 0..S2−1) and accumulates it in registers; the normal stencil is walked as (dy, dx)
// GROUPS, each reading the neighbour column once from LDS and applying its ≤ 5 dt taps to all
// S2 outputs.  Coefficients are stored per (cy, cx) class row × group × t (exact t, padded to
// the template width MAXT with zeros), so the loops are fully unrolled and branch-free.  A
// workgroup streams a strip of ty rows through an LDS ring (lsqr_cg.inc, cg_strip).
constexpr int CG_MAXT = 16;
constexpr int CG_MAX_GRP = 49;
constexpr int CG_NCW = 16;                  // ring staging: row-image columns per lane (a wave stages whole rows: ≤ 1024)
// Node-block factors R_b⁻¹ as the CG update and the multigrid smoother stream them: bf16 (the
// factor was 0.33 of the update's bytes in fp32; its products stay f64).  M⁻¹ = R̃ R̃ᵀ with R̃ the
// rounded upper-triangular R_b⁻¹ (non-zero diagonal) is SPD whatever the rounding, so PCG keeps a
// valid preconditioner; the stopping rule, not M, fixes x.  Packed upper, block stride
// lf_stride(npk) = npk rounded up to a whole 8-byte word.  -DLSQ_LF_F32: the fp32 copy (A/B).
#ifdef LSQ_LF_F32
using lf_t = float;
#else
using lf_t = uint16_t;
#endif
constexpr int LF_PER8 = 8 / (int)sizeof(lf_t);
inline int lf_stride(int npk) { return (npk + LF_PER8 - 1) / LF_PER8 * LF_PER8; }
__device__ __forceinline__ float lf_val(lf_t v) {
#ifdef LSQ_LF_F32
    return v;
#else
    return __uint_as_float((uint32_t)v << 16);
#endif
}
// Column j and row j of a packed block factor (M[r(r+1)/2 + c] = entry (r, c), r ≥ c) with one LDS
// read per entry: fv[i] = (j, i) for i ≤ j, (i, j) for i > j, 0 past the block (k) or off a live
// lane.  The two block products take fv[i] for i ≤ j and for i ≥ j (the diagonal in both).
template <int K>
__device__ __forceinline__ void lf_rowcol(const lf_t* M, int j, int k, bool mine, float (&fv)[K]) {
    const int jj = j * (j + 1) / 2;
#pragma unroll
    for (int i = 0; i < K; ++i) fv[i] = (mine && i < k) ? lf_val(M[i <= j ? jj + i : i * (i + 1) / 2 + j]) : 0.0f;
}
__device__ __forceinline__ lf_t lf_round(double d) {
#ifdef LSQ_LF_F32
    return (float)d;
#else
    uint32_t u = __float_as_uint((float)d);   // round to nearest even on the dropped 16 bits
    u += 0x7fffu + ((u >> 16) & 1u);
    return (lf_t)(u >> 16);
#endif
}

struct CgGrid {
    int32_t shape[3], col0, node0;
    int32_t ty, nty, ntx, tile0;             // tiles of the grid: ids [tile0, tile0 + nty·ntx)
    int32_t hy, hx, ht, tpad, wx;            // halo per dim, LDS dim-2 stride, LDS dim-1 extent
    int32_t front, lds;                      // LDS front pad, doubles of the tile image
    int32_t K[3], ncls[3];                   // boundary classes per dim
    int32_t noff, coef0;                     // normal-stencil offsets, first coefficient
    int32_t loff[CG_MAX_OFF];                // LDS offset of each normal-stencil offset
    int8_t ooff[CG_MAX_OFF][4];              // the offsets (dy, dx, dt)
    FastDiv fd_pad, fd_row;                  // ÷ tpad, ÷ (wx · tpad): staging image index
    FastDiv fd_s2, fd_int;                   // ÷ shape[2], ÷ (CG_TX · shape[2]): interior index
    // column mode
    int32_t maxt, rpw, tq;                   // template column length (1 or CG_MAXT), ring rows per wave and step, -
    int32_t ngrp[3];                         // groups with max |dt| = 0, 1, 2 (stored in that order)
    int32_t rowlen, coefc0;                  // coefficients per (cy, cx) class row; first of this grid
    int32_t gdy[CG_MAX_GRP];                 // dim-0 offset dy of group g
    int32_t gl[CG_MAX_GRP];                  // in-row LDS offset dx·tpad of group g
    int32_t gdx[CG_MAX_GRP];                 // dim-1 offset dx of group g (multigrid tile kernel)
    int32_t gc[CG_MAX_GRP];                  // offset of group g's MAXT × (2·DT_g + 1) coefficients in a row
    // wave-strip operator (lsqr_cg_rw.inc): strips of rw_sx dim-1 positions × rw_ry rows, rw_nsx ×
    // rw_nry of them, rw_chunk per XCD; its class table (per dim-0 class) from coefc[rwc0]
    int32_t rw_sx, rw_nsx, rw_ry, rw_nry, rw_chunk, rwc0;
};
struct BlkAffine {
    int64_t base[16], stride[16];
};
// Normal stencil of one grid on the host: (AᵀA) of the grid's stencil rows as a class table,
// coef[((cy·ncls1 + cx)·ncls2 + ct)·noff + o] = (AᵀA)_{c, c + offs[o]} at every node c of class
// (cy, cx, ct).  Built from the stencil parts (lsqr_cg.inc ns_from_parts) or, on a multigrid
// coarse level, as the Galerkin product PᵀNP of the finer level's table (mg.inc).
struct NsTable {
    bool on = false;
    int shape[3] = {1, 1, 1};
    int K[3] = {0, 0, 0}, ncls[3] = {1, 1, 1};
    int64_t col0 = 0;
    int node0 = 0;
    std::vector<std::array<int, 3>> offs;   // sorted
    std::vector<double> coef;
    const double* row(int cy, int cx, int ct) const {
        return coef.data() + ((size_t)(cy * ncls[1] + cx) * ncls[2] + ct) * offs.size();
    }
};
// A field-valued part on a 2-D grid as the CGNR normal operator applies it (k_cg_var2d): tiles of
// CGV_TY × CGV_TX nodes; t = w·A_v p at the centres of a tile and its halo, q += w·A_vᵀ t and
// Σ t² over the tile's own centres (= pᵀA_vᵀA_v p: each row lives in one tile).
constexpr int CGV_TY = 8, CGV_TX = 64;
struct CgVar {
    int32_t S0, S1, col0, ntpl;
    int32_t lo0, hi0, lo1, hi1;              // centre box (dims 0, 1)
    int32_t nty, ntx, blk0, nfield;          // tiles; first partial slot of this part
    int32_t R, pad;                          // template half-width (1 or 2)
    int32_t oy[MF_MAXT], ox[MF_MAXT], fsel[MF_MAXT];
    double val[MF_MAXT];
    double w;
    int64_t n_eq;
    const double* F;
};
struct MgHier;   // multigrid hierarchy (mg.inc)
void mg_free(MgHier* h);
void mg_graph_drop(MgHier* h);   // its captured replicated-level V-cycle (ranks)
struct CgDesc {
    int32_t n_grids, ntiles, lds_max, colmode;
    int32_t nedge, maxt3, pad[2];            // column mode: workgroups of the CG iteration's k_cg_xedge (pad[0]: <8>;
                                             // pad[1]: lanes per item of the CG iteration's pass, 1 or 8); 3-D column length
    int32_t w8, rw_kt;                       // column mode: the CG iteration runs k_cg_normal_col8 (8-wave workgroups);
                                             // the wave-strip table's dim-2 class width (rw_nc; −1 one row per t)
    int32_t rw, rw_nwg;                      // the wave-strip operator k_cg_normal_rw applies; its workgroups
    CgGrid g[MF_MAX_GRIDS];
};
// CGNR data rows without a stored matrix (lsqr_cg.inc, k_cg_dmf_*): when every interpolation
// grid shares one (y, x) node lattice (and the 3-D ones one t lattice), a data row is fully given
// by its point's float subscripts f_d = (p_d − b0_d)/δ_d (the values lin_op.interp_mtx and
// k_gen_rows derive the weights from) and its row scale.  Points are stored sorted by (y, x)
// cell; cell_ptr gives each cell's run, so AdᵀAd gathers per node without a transpose.
struct DmfDesc {
    int32_t ok, n2, n3, S0, S1, S2;   // 2-D / 3-D parts; lattice shape (S2: t nodes of the 3-D part)
    int64_t npts;
    int64_t col2[2], col3;            // col0 of the 2-D parts' grids and of the 3-D part's grid
};
// PCG-on-AᵀA scalar state (device resident).  Quantities are those of CGLS on A·M^{-1/2}; the
// LSQR estimates (anorm, xnorm of the correction, ‖r‖, ‖Aᵀr‖) follow from the CG scalars through
// the Lanczos relation.
// x is updated every CG_XK-th iteration (round 5; every other one before): the step of phase
// CG_XK − 1 pays x += α_{k−3}p_{k−3} + α_{k−2}p_{k−2} + α_{k−1}p_{k−1} + α_k p_k, the directions of
// the cycle's phases living in CG_XK buffers (CgP) — the update kernel reads x and four p once per
// four steps instead of x and two p every other step (4 B per column and step less)
constexpr int CG_XK = 4;
struct CgP {   // the direction of the cycle's phase i in p[i]
    const double* p[CG_XK];
};
struct CgState {
    double rho, gamma, alpha, beta, alpha_prev, beta_prev;
    double rn2, bnorm, anorm2, pn2, dp, dn2;
    double atol, btol;
    double r1norm, arnorm, xnorm, anorm;
    int64_t itn, maxit;
    int32_t istop, stop, no_stop, pad;
    int32_t pend, pad2;            // steps whose α_k p_k is owed (their phases 0 … pend − 1)
    double pend_a[CG_XK - 1];      // their α
    double anorm_seed;   // lsq_opts.anorm0: the stopping rule's ‖A‖ is max(seed, sqrt(anorm2))
};

struct System {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // column map (Ip_c)
    int64_t n_full = 0, n_keep = 0;
    bool have_colmap = false;
    int64_t n_sorted_rows = 0;   // leading rows ordered by first column in A's SELL copy (data rows)
    DBuf<int32_t> colmap;   // n_full -> compact index or -1

    Csr G, GT;
    DBuf<double> roww;      // m row weights (1 if unset)
    DBuf<uint8_t> rowkeep;  // m (1 keep)
    DBuf<double> rs;        // m effective row scale = roww * keep
    DBuf<double> cs;        // n column scale (preconditioner)
    int cs_mode = -1;       // precond the SELL values were filled with (-1 = stale)
    bool rs_dirty = true;
    Sell A, AT;
    bool sell_built = false;   // A / AT exist (built lazily when the stencil operator is active)
    // Lazy full CSR (structured single-GPU systems): formation stores only the data rows of G
    // (rows [0, npts): Ad, ATd and their values come from them) — the CGNR / LSQR stencil operator,
    // the node-block factors and the constraint-row sums never read the 10⁷–10⁸ stencil rows.  G
    // then keeps G.m = m (logical rows) with npts + 1 row pointers, nnz_full is the formed nnz, and
    // GT is empty until ensure_full_csr() forms both from the generation context kept here (the
    // assembled SELL operator, dense / band factors, lsq_get_csr, lsq_spmv).
    bool g_full = true;
    int64_t nnz_full = 0;
    std::vector<char> gen_ctx;            // GenCtx bytes (assemble.hip)
    DBuf<double> gen_py, gen_px, gen_pt;  // point coordinates of the data rows

    // field-valued stencil parts (lsq_set_stencil_fields): staged by stencil index before the
    // structured formation; the device fields live as long as the matrix (MfPart::F)
    struct StencilFields {
        int32_t stencil = -1, ntpl = 0, nfield = 0;
        int32_t off[MF_MAXT][3] = {};
        double val[MF_MAXT] = {};
        int32_t fsel[MF_MAXT] = {};
        DBuf<double> F;
    };
    std::vector<StencilFields> sfields;
    bool has_var = false;      // the formed operator has field-valued parts

    // structured stencil operator (see MfDesc)
    bool mf = false;
    MfDesc mfh{};
    DBuf<MfDesc> mfd;
    Sell Ad;                   // data rows (SELL, column ids = full ids)
    Csr32 ATd;                 // their transpose: rows = node-enumeration positions, cols = Ad rows
    Csr GdT;                   // transpose of the data rows of G (value source of ATd)
    DBuf<int32_t> keep;        // compact column -> full column
    DBuf<double> csf;          // column scale in the full space (0 = removed column)
    DBuf<double> zv;           // cs ∘ ṽ in the full space (gathered by the stencil rows)

    // block-Jacobi (precond 3): blocks of compact columns (every kept column in exactly one),
    // R_b⁻¹ packed upper-triangular by columns, element e = j(j+1)/2 + i of block b at
    // blk_Ri[b * npk + e], npk = kmax(kmax+1)/2 (a block's factor is one contiguous run: the 16
    // lanes that apply it read it coalesced)
    int64_t nblk = 0;
    int blk_kmax = 0;
    // every block has blk_kmax columns and column j of block b is full id base[j] + b·stride[j]
    // (smooth_fit's node blocks): the CG update computes the ids instead of loading them
    bool blk_affine = false;
    BlkAffine blk_aff{};
    bool blk_user = false;          // blocks came from lsq_set_column_blocks
    DBuf<int64_t> blk_ptr;
    DBuf<int32_t> blk_cols;         // compact ids
    DBuf<int32_t> blk_full;         // full ids (stencil operator v-space)
    DBuf<double> blk_Ri;
    DBuf<double> blk_tab;           // lazily formed systems: the block-diagonal stencil class tables (block.hip)
    bool dist_graph_failed = false; // a rank's batch capture was refused once: eager from then on
    DBuf<lf_t> blk_Lf;              // R_b⁻¹ as CGNR streams it (lf_t, packed upper, block stride lf_stride(npk))
    DBuf<double> blk_tmp;           // structured ranks: block partial sums by column (kmax × n_full) for the halo
    bool blk_valid = false;

    // dense factor (precond 2 / error propagation): R and R⁻¹, npad x npad row-major
    DBuf<double> dR, dRi;
    int64_t dense_ld = 0;
    bool dense_valid = false;

    // band factor (precond 5, band.hip): AᵀA in the column order band_order (empty = natural)
    BandFactor band;
    std::vector<int32_t> band_order;

    // distributed layout (y-slab partition, one rank per GPU): columns [0, n_own) are owned,
    // [n_own, G.n) are ghosts grouped by owner; rows are all owned.  One exchange plan serves
    // the forward halo (owned values -> peers' ghost slots) and the reverse halo (ghost partial
    // sums -> owners, added in peer order).
    bool dist = false;
    bool virt = false;              // in-process virtual rank (shares device + stream with its group)
    bool own_stream = true;
    hipStream_t side = nullptr;              // CGNR: k_cg_xedge beside the data kernel (fork/join events)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipStream_t aux = nullptr, aux_side = nullptr;   // multigrid set-up: coarse power steps beside level 0's
    hipEvent_t ev_aux = nullptr;
    int rank = 0, nranks = 1;
    ncclComm_t comm = nullptr;
    int64_t n_own = 0;
    std::vector<int> peers;
    std::vector<int64_t> send_cnt, send_off, recv_cnt, recv_off;
    DBuf<int32_t> send_idx;         // concatenated by peer: owned local column indices
    DBuf<double> sbuf, rbuf;        // packed forward values / received reverse partials
    DBuf<double> gsum;              // [0] Σu², [1] Σw², [2] Σṽ², [3] Σb² (all-reduced)
    // structured-operator ranks (lsq_dist_set_halo): the local system is the rank's window of
    // node rows (owned rows ± halo rows) on sub-grids; v-space = local full columns; halos move
    // the listed local full ids (send_idx: owned, recv_idx: ghosts), live = owned ∧ kept
    bool dist_mf = false;
    DBuf<int32_t> recv_idx;
    DBuf<uint8_t> live;
    // distributed multigrid (lsq_dist_set_global): the global structure behind a structured rank's
    // window — host description of the global grids and parts (row scales filled per solve), the
    // rank's part of each global part (-1: none), global node rows of the window start and the
    // owned rows [dg_oa, dg_ob), global node rows of the lattice
    bool dg_on = false;
    MfDesc dg_mfh{};
    std::vector<int32_t> dg_local;
    int32_t dg_wa = 0, dg_oa = 0, dg_ob = 0, dg_S0 = 0;
    DBuf<double> dg_w;                 // scratch: the global parts' row scales (all-reduced max)

    // CGNR (method 1): normal-stencil description + coefficient table, rebuilt when the part
    // row scales change; vectors in the full column space
    bool cg_ok = false;            // the structured normal operator exists for this system
    int64_t cg_data_cols = 0;      // columns touched by the data rows
    DmfDesc dmf{};                  // matrix-free data rows for CGNR (ok = 0: use Ad / ATd)
    DBuf<double> dmf_pt;            // per sorted point: f_y, f_x, f_t, row scale (double4)
    DBuf<int32_t> dmf_perm, dmf_cell;   // sorted point -> data row; (y, x) cell -> first sorted point
    std::string cg_why;            // why not (when !cg_ok)
    CgDesc cgh{};
    DBuf<CgDesc> cgd;
    DBuf<double> cg_coef, cg_coefc;  // class-row tables: offset-major (tile mode), group × t (column mode)
    std::vector<NsTable> cg_ns;      // host copy of each grid's normal-stencil table (multigrid input)
    std::vector<CgVar> cg_var;       // field-valued parts (k_cg_var2d), partial slots after the x-edge pass
    int cg_nvb = 0;                  // their workgroups (partial slots)
    MgHier* mg = nullptr;            // precond 4: geometric multigrid levels (mg.inc), built lazily
    // z0 on a 2× refinement of the dz (y, x) lattice (the reference notebooks' z0 50 m / dz 100 m):
    // the multigrid's level 1 is the system Galerkin-projected onto the dz lattice (z0 restricted
    // bilinearly, dz unchanged) — a shared-lattice system with matrix-free data rows (the points
    // sorted by dz cell, z0 interpolated on the dz lattice), held here; mg.inc builds the rest
    System* mx = nullptr;
    int32_t mx_z0col = 0, mx_dzcol = 0, mx_Sf0 = 0, mx_Sf1 = 0, mx_Sc0 = 0, mx_Sc1 = 0, mx_nt = 0;
    std::string mg_why;              // why precond 4 is unavailable
    std::vector<double> cg_wkey;   // part row scales the table was built for
    DBuf<double> cg_x, cg_s, cg_z, cg_q, cg_t, cg_part_g, cg_part_r, cg_part_t;
    DBuf<double> cg_pb[CG_XK];   // the directions of a CG_XK-step cycle (phase i in cg_pb[i])
    DBuf<CgState> cst;
    int cg_parity = 0;
    bool cg_ready = false;         // lsq_iterate state initialised (CG)
    int cg_mode = -1;

    // LSQR workspace
    DBuf<double> u, vb0, vb1, w, y, bw, zt, tt;
    DBuf<double> rhs;          // b of the current solve (persistent: no per-solve allocation)
    DBuf<double> part_u, part_v, part_w, part_b;
    DBuf<LsqState> st;
    bool iter_ready = false;   // lsq_iterate state initialised
    int iter_mode = -1;        // precond * 2 + stencil-operator flag of that state
    int iter_parity = 0;

    int64_t ncols_own() const { return dist ? n_own : G.n; }   // columns whose x this rank solves
    int64_t vlen() const { return mf ? std::max<int64_t>(G.n, n_full) : G.n; }   // workspace v length
    ~System();
};

// A set of ranks solved together.  RCCL mode: the one System of this process (peers live in
// other processes).  Virtual mode: every rank of the problem in this process, on one device and
// one stream, exchanging by device copies — the same kernels and plans, testable on one GPU.
// Host rendezvous of the rank threads of a device group (lsq_dgroup: one thread per device, one
// RCCL communicator each).  Every RCCL call site passes it first, so a rank that fails before a
// collective (an exception on that rank only: a per-rank set-up refusal, a device OOM) poisons the
// fence and the other ranks leave with an error at their next collective instead of blocking in
// it forever.  Spinning: the threads are dedicated to their ranks for the call.
struct GroupFence {
    explicit GroupFence(int n_) : n(n_) {}
    struct Poisoned : std::runtime_error {
        Poisoned() : std::runtime_error("another rank of the device group failed") {}
    };
    void arrive() {
        if (poisoned.load(std::memory_order_acquire)) throw Poisoned();
        const int g = gen.load(std::memory_order_acquire);
        if (count.fetch_add(1, std::memory_order_acq_rel) + 1 == n) {
            count.store(0, std::memory_order_relaxed);
            gen.fetch_add(1, std::memory_order_acq_rel);
            return;
        }
        while (gen.load(std::memory_order_acquire) == g) {
            if (poisoned.load(std::memory_order_acquire)) throw Poisoned();
            std::this_thread::yield();
        }
    }
    // first caller wins: returns true for the rank whose failure is the group's
    bool poison() { return !poisoned.exchange(true, std::memory_order_acq_rel); }
    const int n;
    std::atomic<int> count{0}, gen{0};
    std::atomic<bool> poisoned{false};
};

struct Group {
    std::vector<System*> ranks;
    bool virt = false;
    GroupFence* fence = nullptr;   // device groups: the rank threads' rendezvous before each RCCL call
    DBuf<double*> gs_ptrs;   // virtual all-reduce: device array of the ranks' gsum pointers
    DBuf<double*> vec_ptrs;  // virtual vector all-reduce: the ranks' vector pointers (scratch)
};

inline void group_fence(Group& G) {
    if (G.fence) G.fence->arrive();
}

// dist (build.hip / lsqr.hip)
void group_prepare_virtual(Group& G);
int group_solve(Group& G, const double* const* h_b, double* const* h_x, const lsq_opts& o, lsq_stats* stats);
int group_iterate(Group& G, const double* const* h_b, int64_t iters, const lsq_opts& o, lsq_stats* stats);
int group_cg_solve(Group& G, const double* const* h_b, double* const* h_x, const lsq_opts& o, lsq_stats* stats);
int group_cg_iterate(Group& G, const double* const* h_b, int64_t iters, const lsq_opts& o, lsq_stats* stats);
void referenced_cols(System& S, uint8_t* h_flags);
void relabel_columns(System& S, const int32_t* h_map, int64_t n_local);

// assemble.hip: the full G / GT of a lazily formed structured system (no-op when formed)
void ensure_full_csr(System& S);
bool release_full_csr(System& S);   // back to data rows only (false: not a lazily formed system)
int64_t stored_rows(const System& S);            // rows of G whose entries are stored

// build.hip
void form_from_coo(System& S, int64_t m, int64_t n_full, int64_t nnz, const int64_t* r,
                   const int64_t* c, const double* v);
void finish_formation(System& S);              // G set -> GT, SELL copies, default scaling
void full_transpose(System& S);                 // GT of the (full) G
void describe_global(System& S, int64_t n_full, int32_t n_grids, const lsq_grid_desc* grids, int32_t n_stencil,
                     const lsq_stencil_desc* st);   // S.dg_mfh (lsq_dist_set_global)
void build_dmf(System& S, int32_t n_grids, const lsq_grid_desc* grids, int32_t n_interp, const int32_t* interp_grid,
               int64_t npts, const double* py, const double* px, const double* pt);   // S.dmf (CGNR data rows)
void shape_counts(System& S, int64_t* mk, int64_t* zk);   // assemble.hip: kept rows / entries (lsq_shape)
void ensure_sell(System& S);                    // assembled A / AT (lazy when S.mf)
void refresh_scaling(System& S, int precond);
// band.hip: sqrt(diag((AᵀA)⁻¹)) and op-row variances from a banded Cholesky + Takahashi inverse
void band_factor(System& S, const int32_t* perm, BandFactor& F, int64_t nw = -1);   // nw ≥ 0: a column window
void graph_cache_drop(const System* S);   // lsqr.hip: captured iteration batches of S
void upload_row_mask(System& S, const uint8_t* keep);   // build.hip: rowkeep ← keep (non-zero → 1)
void band_solve_scratch(System& S);
void band_precond(System& S);   // S.band from S.band_order (precond 5)
void band_launch_bsub(System& S, const double* v, int scale_mode, double* out);
void band_launch_fsub(System& S, const double* t, const double* vin, double* vout, double* part);
void band_launch_warm(System& S, const double* x0, double* y0);
void band_check(System& S);   // throws when a precond-5 solve's grid barrier timed out
void band_factor_download(System& S, const int32_t* perm, int64_t* info, double* R_out, double* sc_out,
                          int32_t* perm_out);   // sparseqr.rz drop-in (lsq_band_factor)
// nw ≥ 0 (a window): E in window order (nw entries); inner (nullable): the window positions whose
// tiles are swept (E 0 elsewhere).  nw < 0: E over every compact column.
void band_cov(System& S, const int32_t* perm, int64_t nw, double* E, int64_t nops, const int64_t* rp, const int32_t* ci,
              const double* v, double* op_err, int64_t* info, const uint8_t* inner = nullptr);
// many windows, pipelined over lanes (lsq_cov_band_windows)
void band_cov_windows(System& S, int64_t nwin, const int64_t* win_ptr, const int32_t* perm, const uint8_t* inner,
                      double* E, const int64_t* win_ops, const int64_t* op_ptr, const int32_t* op_pos,
                      const double* op_val, double* op_err, int64_t* info,
                      const int64_t* bot_ptr = nullptr, const int32_t* bot_perm = nullptr,
                      const int64_t* nibs = nullptr);   // rs/cs -> SELL values (single GPU)
void scaling_rows_colnorm(System& S, int precond, bool raw);
void mf_column_scale(System& S, bool raw);       // lsqr.hip: column norms from the stencil structure
void scaling_finish_cs(System& S);
void scaling_fill_values(System& S, int precond, bool set_csf = true);
bool scaling_stale(const System& S, int precond);
void csr_spmv(System& S, int trans, const double* dx, double* dy);  // unweighted G / Gᵀ products
void csr_spmv_rows(System& S, int64_t first, int64_t count, const double* dx, double* dy);
void csr_rows_sumsq(System& S, const double* dx, int64_t first, int64_t count, double* h_w, double* h_u);

// block.hip
void set_column_blocks(System& S, int64_t nb, const int64_t* ptr, const int32_t* cols);
void set_column_blocks_affine(System& S, int64_t nb, int k, const int64_t* base, const int64_t* stride,
                              const int64_t* fbase, const int64_t* fstride);
void ensure_blocks(System& S);                     // default structure if none was set
void block_factor(System& S);                      // R_b⁻¹ for the current row scale
void block_normal(System& S);                      // (AᵀA)_bb of the system's own rows into blk_Ri
void block_factor_in_place(System& S);             // blk_Ri: (AᵀA)_bb -> R_b⁻¹
void block_factor_packed(int64_t nb, const int64_t* ptr, int kmax, double* Ri, lf_t* Lf,
                         unsigned long long* ndead, hipStream_t st);   // multigrid coarse blocks

// dense.hip
void dense_factor(System& S);                     // R, R⁻¹ of diag(rs)·G (throws if not SPD)
void dense_rowrss(System& S, double* dE);         // sqrt(row sums of R⁻¹²) = sqrt(diag((AᵀA)⁻¹))
void dense_spd_factor(double* Nm, double* Ri, int64_t npad, int* err, hipStream_t st);   // multigrid coarsest

// multigrid test hooks (mg.inc; lsq_mg_info / lsq_mg_apply)
int mg_info(System& S, int64_t* out, int64_t cap);
void mg_test_apply(System& S, int level, int what, const double* x, double* y);
__global__ void k_gemv_upper(const double* M, int64_t n, int64_t ld, const double* v, const LsqState* st,
                             int scale_mode, double* z);
__global__ void k_gemvT_upper(const double* M, int64_t n, int64_t ld, const double* t, const LsqState* st, int mode,
                              const double* vin, double* out, double* part);

}  // namespace lsq
