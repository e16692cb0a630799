// api.hip — extern "C" entry points of liblsqsurf.so (declared in include/lsqsurf.h).
#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/lsqsurf.h"
#include "system.hpp"

namespace lsq {
int lsqr_solve(System& S, const double* h_b, double* h_x, const lsq_opts& o, lsq_stats* stats);
bool cg_available(System& S, int precond);
int cg_solve(System& S, const double* h_b, double* h_x, const lsq_opts& o, lsq_stats* stats);
int cg_iterate(System& S, const double* h_b, int64_t iters, const lsq_opts& o, lsq_stats* stats);
void cg_profile(System& S, int reps, int precond, double* out);
void cg_apply_normal(System& S, const double* h_p, double* h_q);
void cg_data_colsum(System& S, const double* h_f, double* h_out);
int lsqr_iterate(System& S, const double* h_b, int64_t iters, const lsq_opts& o, lsq_stats* stats);
void lsqr_profile(System& S, int reps, int op, double* out);
void lsqr_sigma_x(System& S, double* h_E);
void lsqr_get_rinv(System& S, double* h_Ri);
void graph_cache_drop(const System* S);
void form_from_stencils(System& S, int64_t m, int64_t n_full, int32_t n_grids, const lsq_grid_desc* grids,
                        int32_t n_interp, const int32_t* interp_grid, int64_t npts, const double* py,
                        const double* px, const double* pt, int32_t n_stencil, const lsq_stencil_desc* st);
}  // namespace lsq

struct lsq_handle {
    lsq::System sys;
};

namespace {

template <class F>
int guarded(lsq_handle* h, F&& f) {
    if (!h) return -1;
    h->sys.err.clear();
    try {
        HIP_CHECK(hipSetDevice(h->sys.device));
        return f(h->sys);
    } catch (const lsq::Refused& e) {
        h->sys.err = e.what();
        return -5;
    } catch (const std::invalid_argument& e) {
        h->sys.err = e.what();
        return -2;
    } catch (const std::exception& e) {
        h->sys.err = e.what();
        return -3;
    }
}

int fail(lsq::System& S, const std::string& msg) {
    S.err = msg;
    return -2;
}

}  // namespace

extern "C" {

void lsq_default_opts(lsq_opts* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->method = 0;
    o->precond = 1;
    o->atol = 1e-10;
    o->btol = 1e-10;
    o->conlim = 1e8;
    o->maxit = 0;   // 0 -> 4 n
    o->use_x0 = 0;
    o->batch = 16;
    o->use_graph = 1;
}

lsq_handle* lsq_create(int32_t device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return nullptr;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return nullptr;   // gfx950 code objects only
    auto* h = new lsq_handle();
    h->sys.device = device;
    if (hipStreamCreateWithFlags(&h->sys.stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return nullptr;
    }
    return h;
}

void lsq_destroy(lsq_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->sys.device);
    lsq::graph_cache_drop(&h->sys);
    (void)hipStreamSynchronize(h->sys.stream);
    delete h;
}

const char* lsq_last_error(lsq_handle* h) { return h ? h->sys.err.c_str() : "null handle"; }

int lsq_set_col_map(lsq_handle* h, int64_t n_full, const int64_t* keep_cols, int64_t n_keep) {
    return guarded(h, [&](lsq::System& S) {
        if (S.G.rp.p) return fail(S, "lsq_set_col_map must precede lsq_set_matrix_coo");
        if (n_full <= 0 || n_keep < 0 || n_keep > n_full || (n_keep && !keep_cols))
            return fail(S, "lsq_set_col_map: bad sizes");
        std::vector<int32_t> map(n_full, -1);
        for (int64_t k = 0; k < n_keep; ++k) {
            const int64_t c = keep_cols[k];
            if (c < 0 || c >= n_full || (k && c <= keep_cols[k - 1]))
                return fail(S, "lsq_set_col_map: keep_cols must be strictly increasing in [0, n_full)");
            map[c] = (int32_t)k;
        }
        S.colmap.alloc(n_full);
        S.colmap.upload(map.data(), n_full, S.stream);
        HIP_CHECK(hipStreamSynchronize(S.stream));
        S.n_full = n_full;
        S.n_keep = n_keep;
        S.have_colmap = true;
        return 0;
    });
}

int lsq_set_matrix_coo(lsq_handle* h, int64_t m, int64_t n_full, int64_t nnz, const int64_t* r, const int64_t* c,
                       const double* v, const double* row_weight) {
    return guarded(h, [&](lsq::System& S) {
        if (m <= 0 || n_full <= 0 || nnz < 0 || (nnz && (!r || !c || !v)))
            return fail(S, "lsq_set_matrix_coo: bad arguments");
        if (S.have_colmap && n_full != S.n_full) return fail(S, "lsq_set_matrix_coo: n_full differs from col map");
        if (m >= (int64_t)INT32_MAX || n_full >= (int64_t)INT32_MAX)
            return fail(S, "lsq_set_matrix_coo: dimensions must fit int32 column indices");
        if (S.G.rp.p) return fail(S, "lsq_set_matrix_coo: matrix already set (create a new handle)");
        lsq::graph_cache_drop(&S);
        lsq::form_from_coo(S, m, n_full, nnz, r, c, v);
        if (row_weight) {
            S.roww.upload(row_weight, m, S.stream);
            HIP_CHECK(hipStreamSynchronize(S.stream));
        }
        return 0;
    });
}

int lsq_set_matrix_stencil(lsq_handle* h, int64_t m, int64_t n_full, int32_t n_grids, const lsq_grid_desc* grids,
                           int32_t n_interp, const int32_t* interp_grid, int64_t npts, const double* py,
                           const double* px, const double* pt, int32_t n_stencil, const lsq_stencil_desc* stencils,
                           const double* row_weight) {
    return guarded(h, [&](lsq::System& S) {
        if (m <= 0 || n_full <= 0 || npts < 0 || !grids || (n_interp && !interp_grid) || (n_stencil && !stencils))
            return fail(S, "lsq_set_matrix_stencil: bad arguments");
        if (S.have_colmap && n_full != S.n_full) return fail(S, "lsq_set_matrix_stencil: n_full differs from col map");
        if (m >= (int64_t)INT32_MAX || n_full >= (int64_t)INT32_MAX)
            return fail(S, "lsq_set_matrix_stencil: dimensions must fit int32 column indices");
        if (S.G.rp.p) return fail(S, "lsq_set_matrix_stencil: matrix already set (create a new handle)");
        lsq::graph_cache_drop(&S);
        lsq::form_from_stencils(S, m, n_full, n_grids, grids, n_interp, interp_grid, npts, py, px, pt, n_stencil,
                                stencils);
        if (row_weight) {
            S.roww.upload(row_weight, m, S.stream);
            HIP_CHECK(hipStreamSynchronize(S.stream));
        }
        return 0;
    });
}

int lsq_set_stencil_fields(lsq_handle* h, int32_t stencil, int32_t ntpl, const int32_t* off, const double* val,
                           int32_t nfield, const int32_t* fsel, int64_t n_eq, const double* F) {
    return guarded(h, [&](lsq::System& S) {
        if (S.G.rp.p) return fail(S, "lsq_set_stencil_fields must precede lsq_set_matrix_stencil");
        if (stencil < 0 || ntpl < 1 || ntpl > lsq::MF_MAXT || !off || !val || nfield < 1 || nfield > ntpl || !fsel ||
            n_eq < 0 || (n_eq && !F))
            return fail(S, "lsq_set_stencil_fields: bad arguments");
        for (int t = 0; t < ntpl; ++t)
            if (fsel[t] < 0 || fsel[t] >= nfield) return fail(S, "lsq_set_stencil_fields: fsel out of range");
        S.sfields.erase(std::remove_if(S.sfields.begin(), S.sfields.end(),
                                       [&](const lsq::System::StencilFields& f) { return f.stencil == stencil; }),
                        S.sfields.end());
        lsq::System::StencilFields f;
        f.stencil = stencil;
        f.ntpl = ntpl;
        f.nfield = nfield;
        for (int t = 0; t < ntpl; ++t) {
            for (int d = 0; d < 3; ++d) f.off[t][d] = off[3 * t + d];
            f.val[t] = val[t];
            f.fsel[t] = fsel[t];
        }
        f.F.alloc(std::max<int64_t>((int64_t)nfield * n_eq, 1));
        f.F.upload(F, (int64_t)nfield * n_eq, S.stream);
        HIP_CHECK(hipStreamSynchronize(S.stream));
        S.sfields.push_back(std::move(f));
        return 0;
    });
}

int lsq_set_row_weight(lsq_handle* h, const double* row_weight) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_set_row_weight: no matrix");
        if (row_weight) {
            S.roww.upload(row_weight, S.G.m, S.stream);
        } else {
            std::vector<double> one(S.G.m, 1.0);
            S.roww.upload(one.data(), S.G.m, S.stream);
        }
        HIP_CHECK(hipStreamSynchronize(S.stream));
        S.rs_dirty = true;
        return 0;
    });
}

int lsq_set_column_blocks(lsq_handle* h, int64_t n_blocks, const int64_t* block_ptr, const int32_t* cols) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_set_column_blocks: no matrix");
        if (S.dist && !S.dist_mf) return fail(S, "lsq_set_column_blocks: single-GPU or structured-rank handles only");
        lsq::graph_cache_drop(&S);
        lsq::set_column_blocks(S, n_blocks > 0 ? n_blocks : 0, block_ptr, cols);
        return 0;
    });
}

int lsq_set_column_blocks_affine(lsq_handle* h, int64_t n_blocks, int32_t k, const int64_t* base,
                                 const int64_t* stride, const int64_t* full_base, const int64_t* full_stride) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_set_column_blocks_affine: no matrix");
        if (S.dist) return fail(S, "lsq_set_column_blocks_affine: single-GPU handles only");
        lsq::graph_cache_drop(&S);
        lsq::set_column_blocks_affine(S, n_blocks, k, base, stride, full_base, full_stride);
        return 0;
    });
}

int lsq_set_row_mask(lsq_handle* h, const uint8_t* keep) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_set_row_mask: no matrix");
        lsq::upload_row_mask(S, keep);
        S.rs_dirty = true;
        return 0;
    });
}

int lsq_shape(lsq_handle* h, int64_t* m, int64_t* n, int64_t* nnz) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_shape: no matrix");
        int64_t mk = 0, zk = 0;
        lsq::shape_counts(S, &mk, &zk);   // no full CSR formed for it
        if (m) *m = mk;
        if (n) *n = S.G.n;
        if (nnz) *nnz = zk;
        return 0;
    });
}

int lsq_release_full_csr(lsq_handle* h, int32_t* released) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_release_full_csr: no matrix");
        const bool r = lsq::release_full_csr(S);
        if (released) *released = r ? 1 : 0;
        return 0;
    });
}

int lsq_get_csr(lsq_handle* h, int64_t* indptr, int32_t* indices, double* data) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_get_csr: no matrix");
        lsq::ensure_full_csr(S);
        const int64_t m = S.G.m, z = S.G.nnz;
        std::vector<int64_t> rp(m + 1);
        std::vector<int32_t> ci(std::max<int64_t>(z, 1));
        std::vector<double> val(std::max<int64_t>(z, 1)), rw(m);
        std::vector<uint8_t> keep(m);
        S.G.rp.download(rp.data(), m + 1, S.stream);
        S.G.ci.download(ci.data(), z, S.stream);
        S.G.val.download(val.data(), z, S.stream);
        S.roww.download(rw.data(), m, S.stream);
        S.rowkeep.download(keep.data(), m, S.stream);
        HIP_CHECK(hipStreamSynchronize(S.stream));
        int64_t o = 0, r = 0;
        indptr[0] = 0;
        for (int64_t i = 0; i < m; ++i) {
            if (!keep[i]) continue;
            for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
                indices[o] = ci[e];
                data[o] = val[e] * rw[i];   // = TCinv·G entry, the single IEEE product the reference forms
                ++o;
            }
            indptr[++r] = o;
        }
        return 0;
    });
}

int lsq_solve(lsq_handle* h, const double* b, double* x_inout, const lsq_opts* o, lsq_stats* s) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_solve: no matrix");
        if (!b || !x_inout) return fail(S, "lsq_solve: null b or x");
        lsq_opts d;
        lsq_default_opts(&d);
        if (!o) o = &d;
        if (o->method != 0 && o->method != 1) return fail(S, "lsq_solve: method must be 0 (LSQR) or 1 (CGNR)");
        if (o->precond < 0 || o->precond > 5) return fail(S, "lsq_solve: precond must be 0 .. 5");
        if (o->precond == 5 && S.dist) return fail(S, "lsq_solve: precond 5 (band factor) is single-GPU");
        if (o->precond == 4 && (o->method != 1 || (!S.dist && !lsq::cg_available(S, 4))))
            return fail(S, "lsq_solve: precond 4 (multigrid) runs CGNR (method 1) on structured systems: " +
                               (o->method != 1 ? std::string("method is not 1") : S.cg_ok ? S.mg_why : S.cg_why));
        if (S.dist) {
            if (S.virt) return fail(S, "lsq_solve: a virtual rank solves through lsq_vgroup_solve");
            lsq::Group G;
            G.ranks = {&S};
            double* xs[1] = {x_inout};
            return o->method == 1 ? lsq::group_cg_solve(G, &b, xs, *o, s) : lsq::group_solve(G, &b, xs, *o, s);
        }
        const auto t_prep = std::chrono::steady_clock::now();
        if (o->method == 1 && lsq::cg_available(S, o->precond)) {   // builds block factors / levels when stale
            HIP_CHECK(hipStreamSynchronize(S.stream));
            const double prep_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_prep).count();
            if (getenv("LSQ_SETUP_TRACE")) fprintf(stderr, "setup %-16s %8.3f ms\n", "prepare", prep_s * 1e3);
            const int rc = lsq::cg_solve(S, b, x_inout, *o, s);
            if (s) s->setup_s += prep_s;
            return rc;
        }
        if (s) {
            s->method = 0;
            s->setup_s = 0.0;
        }
        return lsq::lsqr_solve(S, b, x_inout, *o, s);
    });
}

int lsq_iterate(lsq_handle* h, const double* b, int64_t iters, const lsq_opts* o, lsq_stats* s) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_iterate: no matrix");
        lsq_opts d;
        lsq_default_opts(&d);
        if (!o) o = &d;
        if (o->precond == 4 && (o->method != 1 || (!S.dist && !lsq::cg_available(S, 4))))
            return fail(S, "lsq_iterate: precond 4 (multigrid) runs CGNR (method 1) on structured systems: " +
                               (o->method != 1 ? std::string("method is not 1") : S.cg_ok ? S.mg_why : S.cg_why));
        if (S.dist) {
            if (S.virt) return fail(S, "lsq_iterate: a virtual rank iterates through lsq_vgroup_iterate");
            lsq::Group G;
            G.ranks = {&S};
            return o->method == 1 ? lsq::group_cg_iterate(G, &b, iters, *o, s) : lsq::group_iterate(G, &b, iters, *o, s);
        }
        if (o->method == 1 && lsq::cg_available(S, o->precond)) return lsq::cg_iterate(S, b, iters, *o, s);
        if (s) s->method = 0;
        return lsq::lsqr_iterate(S, b, iters, *o, s);
    });
}

int lsq_cg_available(lsq_handle* h, int32_t precond) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_cg_available: no matrix");
        if (precond != 1 && precond != 3 && precond != 4) {
            S.err = "CGNR runs with precond 1 (Jacobi), 3 (block-Jacobi) or 4 (multigrid)";
            return 0;
        }
        if (lsq::cg_available(S, precond)) return 1;
        S.err = !S.cg_ok ? (S.cg_why.empty() ? "not a structured single-GPU system" : S.cg_why) : S.mg_why;
        return 0;
    });
}

int lsq_profile_cg(lsq_handle* h, int32_t reps, int32_t precond, double* out8) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_profile_cg: no matrix");
        if (!out8) return fail(S, "lsq_profile_cg: null output");
        if (!lsq::cg_available(S, precond)) return fail(S, "lsq_profile_cg: CGNR not available: " + S.cg_why);
        lsq::graph_cache_drop(&S);
        lsq::cg_profile(S, reps > 0 ? reps : 10, precond, out8);
        return 0;
    });
}

int lsq_mg_info(lsq_handle* h, int64_t* out, int64_t cap) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_mg_info: no matrix");
        if (!out) return fail(S, "lsq_mg_info: null output");
        return lsq::mg_info(S, out, cap);
    });
}

int lsq_mg_apply(lsq_handle* h, int32_t level, int32_t what, const double* x, double* y) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_mg_apply: no matrix");
        if (!y || (what != 2 && !x)) return fail(S, "lsq_mg_apply: null vector");
        lsq::mg_test_apply(S, level, what, x, y);
        return 0;
    });
}

int lsq_normal_apply(lsq_handle* h, const double* p, double* q) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_normal_apply: no matrix");
        if (!p || !q) return fail(S, "lsq_normal_apply: null vector");
        if (!lsq::cg_available(S, 1)) return fail(S, "lsq_normal_apply: no normal-stencil operator: " + S.cg_why);
        lsq::cg_apply_normal(S, p, q);
        return 0;
    });
}

int lsq_profile_kernels(lsq_handle* h, int32_t reps, int32_t op, double* out8) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_profile_kernels: no matrix");
        if (!out8) return fail(S, "lsq_profile_kernels: null output");
        lsq::graph_cache_drop(&S);
        lsq::lsqr_profile(S, reps > 0 ? reps : 10, op, out8);
        return 0;
    });
}

int lsq_sell_info(lsq_handle* h, int64_t* out8) {
    return guarded(h, [&](lsq::System& S) {
        if (!out8) return fail(S, "lsq_sell_info: null output");
        out8[0] = S.G.m;
        out8[1] = S.G.n;
        out8[2] = S.g_full ? S.G.nnz : S.nnz_full;   // the formed operator's nnz
        out8[3] = S.mf ? S.Ad.nent : S.A.nent;
        out8[4] = S.mf ? S.ATd.nnz : S.AT.nent;
        out8[5] = (int64_t)(S.G.rp.bytes() + S.G.ci.bytes() + S.G.val.bytes() + S.GT.rp.bytes() + S.GT.ci.bytes() +
                            S.GT.val.bytes() + S.A.ci.bytes() + S.A.val.bytes() + S.AT.ci.bytes() + S.AT.val.bytes() +
                            S.Ad.ci.bytes() + S.Ad.val.bytes() + S.ATd.ci.bytes() + S.ATd.val.bytes() +
                            S.GdT.ci.bytes() + S.GdT.val.bytes());
        out8[6] = S.mf ? 1 : 0;
        out8[7] = S.n_full;
        return 0;
    });
}

int lsq_dist_unique_id(uint8_t* id) {
    if (!id) return -1;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return -3;
    std::memcpy(id, &u, sizeof(u));
    return 0;
}

lsq_handle* lsq_create_dist(int32_t device, int32_t rank, int32_t nranks, const uint8_t* id) {
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) return nullptr;
    lsq_handle* h = lsq_create(device);
    if (!h) return nullptr;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    if (ncclCommInitRank(&h->sys.comm, nranks, u, rank) != ncclSuccess) {
        h->sys.comm = nullptr;
        lsq_destroy(h);
        return nullptr;
    }
    h->sys.rank = rank;
    h->sys.nranks = nranks;
    return h;
}

int lsq_dist_comm_info(lsq_handle* h, int64_t* out) {
    return guarded(h, [&](lsq::System& S) {
        if (!out) return fail(S, "lsq_dist_comm_info: null output");
        for (int k = 0; k < 7; ++k) out[k] = 0;
        if (S.comm) {
            int c = 0, r = 0, d = 0;
            if (ncclCommCount(S.comm, &c) != ncclSuccess || ncclCommUserRank(S.comm, &r) != ncclSuccess ||
                ncclCommCuDevice(S.comm, &d) != ncclSuccess)
                return fail(S, "lsq_dist_comm_info: RCCL query failed");
            out[0] = c;
            out[1] = r;
            out[2] = d;
        }
        out[3] = S.device;
        int v = 0;
        HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributePciDomainID, S.device));
        out[4] = v;
        HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributePciBusId, S.device));
        out[5] = v;
        HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributePciDeviceId, S.device));
        out[6] = v;
        return 0;
    });
}

int lsq_dist_referenced_cols(lsq_handle* h, uint8_t* flags) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p || !flags) return fail(S, "lsq_dist_referenced_cols: no matrix / null output");
        if (S.dist) return fail(S, "lsq_dist_referenced_cols: layout already set");
        lsq::referenced_cols(S, flags);
        return 0;
    });
}

int lsq_dist_set_layout(lsq_handle* h, const int32_t* col_local, int64_t n_local, int64_t n_own, int32_t n_peers,
                        const int32_t* peers, const int64_t* send_cnt, const int32_t* send_idx,
                        const int64_t* recv_cnt) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.comm && !S.virt)
            return fail(S, "lsq_dist_set_layout: handle has no communicator (use lsq_create_dist / lsq_vgroup)");
        if (!S.G.rp.p || S.dist) return fail(S, "lsq_dist_set_layout: needs a formed matrix, once");
        if (!col_local || n_own < 0 || n_own > n_local || n_peers < 0) return fail(S, "lsq_dist_set_layout: bad args");
        S.peers.assign(peers, peers + n_peers);
        S.send_cnt.assign(send_cnt, send_cnt + n_peers);
        S.recv_cnt.assign(recv_cnt, recv_cnt + n_peers);
        S.send_off.assign(n_peers, 0);
        S.recv_off.assign(n_peers, 0);
        int64_t ts = 0, tr = 0;
        for (int k = 0; k < n_peers; ++k) {
            if (peers[k] < 0 || peers[k] >= S.nranks || peers[k] == S.rank)
                return fail(S, "lsq_dist_set_layout: bad peer rank");
            S.send_off[k] = ts;
            S.recv_off[k] = tr;
            ts += send_cnt[k];
            tr += recv_cnt[k];
        }
        if (tr != n_local - n_own) return fail(S, "lsq_dist_set_layout: receive counts must cover the ghosts");
        for (int64_t k = 0; k < ts; ++k)
            if (send_idx[k] < 0 || send_idx[k] >= n_own) return fail(S, "lsq_dist_set_layout: send index not owned");
        lsq::graph_cache_drop(&S);
        lsq::relabel_columns(S, col_local, n_local);
        S.n_own = n_own;
        S.send_idx.alloc(ts);
        S.send_idx.upload(send_idx, ts, S.stream);
        S.sbuf.alloc(std::max<int64_t>(ts, 1));
        S.rbuf.alloc(std::max<int64_t>(ts, 1));
        S.gsum.alloc(16);
        S.gsum.zero(S.stream);
        HIP_CHECK(hipStreamSynchronize(S.stream));
        S.dist = true;
        S.u = lsq::DBuf<double>();
        S.vb0 = lsq::DBuf<double>();   // workspace re-sized on first use
        return 0;
    });
}

int lsq_dist_set_halo(lsq_handle* h, int32_t n_ranges, const int64_t* own_ranges, int32_t n_peers,
                      const int32_t* peers, const int64_t* send_cnt, const int32_t* send_idx,
                      const int64_t* recv_cnt, const int32_t* recv_idx) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.comm && !S.virt)
            return fail(S, "lsq_dist_set_halo: handle has no communicator (use lsq_create_dist / lsq_vgroup)");
        if (!S.G.rp.p || S.dist) return fail(S, "lsq_dist_set_halo: needs a formed matrix, once");
        if (!S.mf) return fail(S, "lsq_dist_set_halo: needs a structured system (lsq_set_matrix_stencil)");
        if (n_ranges < 0 || (n_ranges && !own_ranges) || n_peers < 0) return fail(S, "lsq_dist_set_halo: bad args");
        const int64_t nf = S.n_full;
        std::vector<uint8_t> own(nf, 0);
        for (int i = 0; i < n_ranges; ++i) {
            const int64_t a = own_ranges[2 * i], b = own_ranges[2 * i + 1];
            if (a < 0 || b > nf || a > b) return fail(S, "lsq_dist_set_halo: owned range outside the local columns");
            std::fill(own.begin() + a, own.begin() + b, 1);
        }
        S.peers.assign(peers, peers + n_peers);
        S.send_cnt.assign(send_cnt, send_cnt + n_peers);
        S.recv_cnt.assign(recv_cnt, recv_cnt + n_peers);
        S.send_off.assign(n_peers, 0);
        S.recv_off.assign(n_peers, 0);
        int64_t ts = 0, tr = 0;
        for (int k = 0; k < n_peers; ++k) {
            if (peers[k] < 0 || peers[k] >= S.nranks || peers[k] == S.rank)
                return fail(S, "lsq_dist_set_halo: bad peer rank");
            S.send_off[k] = ts;
            S.recv_off[k] = tr;
            ts += send_cnt[k];
            tr += recv_cnt[k];
        }
        for (int64_t k = 0; k < ts; ++k)
            if (send_idx[k] < 0 || send_idx[k] >= nf || !own[send_idx[k]])
                return fail(S, "lsq_dist_set_halo: send index not an owned local column");
        for (int64_t k = 0; k < tr; ++k)
            if (recv_idx[k] < 0 || recv_idx[k] >= nf || own[recv_idx[k]])
                return fail(S, "lsq_dist_set_halo: receive index not a ghost local column");
        // live = owned and kept (Ip_c)
        std::vector<int32_t> keep(S.G.n);
        S.keep.download(keep.data(), S.G.n, S.stream);
        HIP_CHECK(hipStreamSynchronize(S.stream));
        std::vector<uint8_t> live(nf, 0);
        for (int32_t f : keep) live[f] = own[f];
        lsq::graph_cache_drop(&S);
        S.live.alloc(std::max<int64_t>(nf, 1));
        S.live.upload(live.data(), nf, S.stream);
        S.send_idx.alloc(std::max<int64_t>(ts, 1));
        S.send_idx.upload(send_idx, ts, S.stream);
        S.send_idx.n = ts;
        S.recv_idx.alloc(std::max<int64_t>(tr, 1));
        S.recv_idx.upload(recv_idx, tr, S.stream);
        S.recv_idx.n = tr;
        const int64_t nb = std::max<int64_t>(std::max(ts, tr), 1);
        S.sbuf.alloc(nb);
        S.rbuf.alloc(nb);
        S.gsum.alloc(16);
        S.gsum.zero(S.stream);
        HIP_CHECK(hipStreamSynchronize(S.stream));
        S.n_own = S.G.n;
        S.dist = true;
        S.dist_mf = true;
        S.cs_mode = -1;
        S.iter_ready = false;
        return 0;
    });
}

int lsq_sigma_x(lsq_handle* h, double* E) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_sigma_x: no matrix");
        if (!E) return fail(S, "lsq_sigma_x: null output");
        lsq::lsqr_sigma_x(S, E);
        return 0;
    });
}

int lsq_set_band_order(lsq_handle* h, int64_t n, const int32_t* perm) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_set_band_order: no matrix");
        if (perm && n != S.G.n) return fail(S, "lsq_set_band_order: the order needs one entry per column");
        std::vector<char> seen(perm ? n : 0, 0);
        for (int64_t j = 0; perm && j < n; ++j) {
            if (perm[j] < 0 || perm[j] >= n || seen[perm[j]]) return fail(S, "lsq_set_band_order: not a permutation");
            seen[perm[j]] = 1;
        }
        S.band_order.assign(perm ? perm : nullptr, perm ? perm + n : nullptr);
        S.band.valid = false;
        S.iter_ready = false;
        return 0;
    });
}

int lsq_cov_band(lsq_handle* h, const int32_t* perm, double* E, int64_t n_ops, const int64_t* op_ptr,
                 const int32_t* op_col, const double* op_val, double* op_err, int64_t* info) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_cov_band: no matrix");
        if (S.dist) return fail(S, "lsq_cov_band: not available on distributed handles");
        if (!E) return fail(S, "lsq_cov_band: null output");
        if (n_ops < 0 || (n_ops > 0 && (!op_ptr || !op_err || (op_ptr[n_ops] > 0 && (!op_col || !op_val)))))
            return fail(S, "lsq_cov_band: bad op rows");
        lsq::band_cov(S, perm, -1, E, n_ops, op_ptr, op_col, op_val, op_err, info);
        return 0;
    });
}

int lsq_cov_band_window(lsq_handle* h, const int32_t* perm, int64_t n_win, const uint8_t* inner, double* E,
                        int64_t n_ops, const int64_t* op_ptr, const int32_t* op_col, const double* op_val,
                        double* op_err, int64_t* info) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_cov_band_window: no matrix");
        if (S.dist) return fail(S, "lsq_cov_band_window: not available on distributed handles");
        if (!E || !perm || n_win < 1 || n_win > S.G.n) return fail(S, "lsq_cov_band_window: bad window");
        if (n_ops < 0 || (n_ops > 0 && (!op_ptr || !op_err || (op_ptr[n_ops] > 0 && (!op_col || !op_val)))))
            return fail(S, "lsq_cov_band_window: bad op rows");
        lsq::band_cov(S, perm, n_win, E, n_ops, op_ptr, op_col, op_val, op_err, info, inner);
        return 0;
    });
}

int lsq_cov_band_windows(lsq_handle* h, int64_t n_windows, const int64_t* win_ptr, const int32_t* perm,
                         const uint8_t* inner, double* E, const int64_t* win_ops, const int64_t* op_ptr,
                         const int32_t* op_pos, const double* op_val, double* op_err, int64_t* info) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_cov_band_windows: no matrix");
        if (S.dist) return fail(S, "lsq_cov_band_windows: not available on distributed handles");
        if (n_windows < 1 || !win_ptr || !perm || !E || win_ptr[0] != 0)
            return fail(S, "lsq_cov_band_windows: bad windows");
        if (win_ops && (!op_ptr || !op_err || (op_ptr[win_ops[n_windows]] > 0 && (!op_pos || !op_val))))
            return fail(S, "lsq_cov_band_windows: bad op rows");
        lsq::band_cov_windows(S, n_windows, win_ptr, perm, inner, E, win_ops, op_ptr, op_pos, op_val, op_err, info);
        return 0;
    });
}

int lsq_cov_band_windows_schur(lsq_handle* h, int64_t n_windows, const int64_t* win_ptr, const int32_t* perm,
                               const uint8_t* inner, double* E, const int64_t* bot_ptr, const int32_t* bot_perm,
                               const int64_t* nib, int64_t* info) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_cov_band_windows_schur: no matrix");
        if (S.dist) return fail(S, "lsq_cov_band_windows_schur: not available on distributed handles");
        if (n_windows < 1 || !win_ptr || !perm || !E || win_ptr[0] != 0 || !bot_ptr || bot_ptr[0] != 0 || !nib ||
            (bot_ptr[n_windows] > 0 && !bot_perm))
            return fail(S, "lsq_cov_band_windows_schur: bad windows");
        for (int64_t w = 0; w < n_windows; ++w)
            for (int64_t j = bot_ptr[w]; j < bot_ptr[w + 1]; ++j)
                if (bot_perm[j] < 0 || bot_perm[j] >= S.G.n) return fail(S, "lsq_cov_band_windows_schur: column out of range");
        lsq::band_cov_windows(S, n_windows, win_ptr, perm, inner, E, nullptr, nullptr, nullptr, nullptr, nullptr, info,
                              bot_ptr, bot_perm, nib);
        return 0;
    });
}

int lsq_dist_set_global(lsq_handle* h, int64_t n_full, int32_t n_grids, const lsq_grid_desc* grids, int32_t n_stencil,
                        const lsq_stencil_desc* stencils, const int32_t* local_of, int32_t win_row0, int32_t own_row0,
                        int32_t own_row1, int32_t rows) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.dist_mf) return fail(S, "lsq_dist_set_global: needs a structured rank (lsq_dist_set_halo first)");
        if (!grids || (n_stencil && (!stencils || !local_of)) || own_row0 < 0 || own_row1 <= own_row0 || win_row0 < 0 ||
            win_row0 > own_row0 || rows < own_row1)
            return fail(S, "lsq_dist_set_global: bad arguments");
        lsq::describe_global(S, n_full, n_grids, grids, n_stencil, stencils);
        S.dg_local.clear();
        for (int s = 0; s < n_stencil; ++s) {
            if (stencils[s].n_eq == 0) continue;
            if (local_of[s] >= S.mfh.n_parts) return fail(S, "lsq_dist_set_global: local part out of range");
            S.dg_local.push_back(local_of[s]);
        }
        S.dg_wa = win_row0;
        S.dg_oa = own_row0;
        S.dg_ob = own_row1;
        S.dg_S0 = rows;
        S.dg_on = true;
        lsq::graph_cache_drop(&S);
        lsq::mg_free(S.mg);
        S.mg = nullptr;
        S.mg_why.clear();
        return 0;
    });
}

int lsq_band_factor(lsq_handle* h, const int32_t* perm, int64_t* info, double* R, double* sc, int32_t* perm_out) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_band_factor: no matrix");
        if (S.dist) return fail(S, "lsq_band_factor: not available on distributed handles");
        if (!info) return fail(S, "lsq_band_factor: null info");
        lsq::band_factor_download(S, perm, info, R, sc, perm_out);
        return 0;
    });
}

int lsq_get_rinv(lsq_handle* h, double* Rinv) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_get_rinv: no matrix");
        if (!Rinv) return fail(S, "lsq_get_rinv: null output");
        lsq::lsqr_get_rinv(S, Rinv);
        return 0;
    });
}

int lsq_spmv(lsq_handle* h, int32_t trans, const double* x, double* y) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_spmv: no matrix");
        const int64_t nin = trans ? S.G.m : S.G.n, nout = trans ? S.G.n : S.G.m;
        lsq::DBuf<double> dx(std::max<int64_t>(nin, 1)), dy(std::max<int64_t>(nout, 1));
        dx.upload(x, nin, S.stream);
        lsq::csr_spmv(S, trans ? 1 : 0, dx.p, dy.p);
        dy.download(y, nout, S.stream);
        HIP_CHECK(hipStreamSynchronize(S.stream));
        return 0;
    });
}

int lsq_spmv_rows(lsq_handle* h, int64_t first, int64_t count, const double* x, double* y) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_spmv_rows: no matrix");
        if (first < 0 || count < 0 || first + count > S.G.m) return fail(S, "lsq_spmv_rows: rows out of range");
        lsq::DBuf<double> dx(std::max<int64_t>(S.G.n, 1)), dy(std::max<int64_t>(count, 1));
        dx.upload(x, S.G.n, S.stream);
        lsq::csr_spmv_rows(S, first, count, dx.p, dy.p);
        dy.download(y, count, S.stream);
        HIP_CHECK(hipStreamSynchronize(S.stream));
        return 0;
    });
}

int lsq_rows_sumsq(lsq_handle* h, const double* x, int32_t n_ranges, const int64_t* first, const int64_t* count,
                   double* sum_w, double* sum_u) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_rows_sumsq: no matrix");
        if (!x || n_ranges < 0 || (n_ranges && (!first || !count || !sum_w || !sum_u)))
            return fail(S, "lsq_rows_sumsq: null argument");
        for (int32_t k = 0; k < n_ranges; ++k)
            if (first[k] < 0 || count[k] < 0 || first[k] + count[k] > S.G.m) return fail(S, "lsq_rows_sumsq: rows out of range");
        lsq::DBuf<double> dx(std::max<int64_t>(S.G.n, 1));
        dx.upload(x, S.G.n, S.stream);
        for (int32_t k = 0; k < n_ranges; ++k) lsq::csr_rows_sumsq(S, dx.p, first[k], count[k], sum_w + k, sum_u + k);
        return 0;
    });
}

int lsq_data_colsum(lsq_handle* h, const double* f, double* out) {
    return guarded(h, [&](lsq::System& S) {
        if (!S.G.rp.p) return fail(S, "lsq_data_colsum: no matrix");
        if (!f || !out) return fail(S, "lsq_data_colsum: null argument");
        lsq::cg_data_colsum(S, f, out);
        return 0;
    });
}

struct lsq_vgroup {
    std::vector<lsq_handle*> h;
    hipStream_t stream = nullptr;
    lsq::Group G;
    std::string err;
};

lsq_vgroup* lsq_vgroup_create(int32_t device, int32_t nranks) {
    if (nranks < 1) return nullptr;
    auto* g = new lsq_vgroup();
    for (int r = 0; r < nranks; ++r) {
        lsq_handle* h = lsq_create(device);
        if (!h) {
            lsq_vgroup_destroy(g);
            return nullptr;
        }
        h->sys.virt = true;
        h->sys.rank = r;
        h->sys.nranks = nranks;
        if (r == 0) {
            g->stream = h->sys.stream;
        } else {   // every virtual rank runs on rank 0's stream: exchanges need no extra sync
            (void)hipStreamDestroy(h->sys.stream);
            h->sys.stream = g->stream;
            h->sys.own_stream = false;
        }
        g->h.push_back(h);
    }
    return g;
}

lsq_handle* lsq_vgroup_rank(lsq_vgroup* g, int32_t rank) {
    return (g && rank >= 0 && rank < (int)g->h.size()) ? g->h[rank] : nullptr;
}

const char* lsq_vgroup_last_error(lsq_vgroup* g) { return g ? g->err.c_str() : "null group"; }

void lsq_vgroup_destroy(lsq_vgroup* g) {
    if (!g) return;
    for (int r = (int)g->h.size() - 1; r >= 0; --r) lsq_destroy(g->h[r]);   // rank 0 owns the stream
    delete g;
}

}  // extern "C"

template <class F>
static int vguarded(lsq_vgroup* g, F&& f) {
    if (!g || g->h.empty()) return -1;
    g->err.clear();
    try {
        HIP_CHECK(hipSetDevice(g->h[0]->sys.device));
        if (g->G.ranks.empty()) {
            for (auto* h : g->h) {
                if (!h->sys.dist) throw std::invalid_argument("every virtual rank needs lsq_dist_set_layout first");
                g->G.ranks.push_back(&h->sys);
            }
            g->G.virt = true;
            lsq::group_prepare_virtual(g->G);
        }
        return f(g->G);
    } catch (const std::invalid_argument& e) {
        g->err = e.what();
        return -2;
    } catch (const std::exception& e) {
        g->err = e.what();
        return -3;
    }
}

extern "C" {

int lsq_vgroup_solve(lsq_vgroup* g, const double* const* b, double* const* x, const lsq_opts* o, lsq_stats* s) {
    return vguarded(g, [&](lsq::Group& G) {
        lsq_opts d;
        lsq_default_opts(&d);
        const lsq_opts& oo = o ? *o : d;
        return oo.method == 1 ? lsq::group_cg_solve(G, b, x, oo, s) : lsq::group_solve(G, b, x, oo, s);
    });
}

int lsq_vgroup_iterate(lsq_vgroup* g, const double* const* b, int64_t iters, const lsq_opts* o, lsq_stats* s) {
    return vguarded(g, [&](lsq::Group& G) {
        lsq_opts d;
        lsq_default_opts(&d);
        const lsq_opts& oo = o ? *o : d;
        return oo.method == 1 ? lsq::group_cg_iterate(G, b, iters, oo, s) : lsq::group_iterate(G, b, iters, oo, s);
    });
}

}  // extern "C"

// ---- device group: N devices driven from one process (smooth_fit(n_gpus=N)) ------------------
// One RCCL communicator per device (ncclCommInitAll) and, per solve, one host thread per device
// running that rank's solve exactly as a one-process-per-GPU rank does (Group of one rank: the
// same kernels, halos and all-reduces).  The ranks are invisible to the caller.
struct lsq_dgroup {
    std::vector<lsq_handle*> h;
    std::string err;
};
// (the rank threads of one call meet at an lsq::GroupFence before every RCCL call: dgroup_run)

extern "C" {

lsq_dgroup* lsq_dgroup_create(int32_t n, const int32_t* devices) {
    if (n < 1 || !devices) return nullptr;
    for (int a = 0; a < n; ++a)
        for (int b = 0; b < a; ++b)
            if (devices[a] == devices[b]) return nullptr;   // RCCL: one rank per device (tests: lsq_vgroup)
    auto* g = new lsq_dgroup();
    for (int r = 0; r < n; ++r) {
        lsq_handle* h = lsq_create(devices[r]);
        if (!h) {
            lsq_dgroup_destroy(g);
            return nullptr;
        }
        h->sys.rank = r;
        h->sys.nranks = n;
        g->h.push_back(h);
    }
    std::vector<ncclComm_t> comms(n, nullptr);
    std::vector<int> devs(devices, devices + n);
    if (ncclCommInitAll(comms.data(), n, devs.data()) != ncclSuccess) {
        lsq_dgroup_destroy(g);
        return nullptr;
    }
    for (int r = 0; r < n; ++r) g->h[r]->sys.comm = comms[r];
    return g;
}

lsq_handle* lsq_dgroup_rank(lsq_dgroup* g, int32_t rank) {
    return (g && rank >= 0 && rank < (int)g->h.size()) ? g->h[rank] : nullptr;
}

const char* lsq_dgroup_last_error(lsq_dgroup* g) { return g ? g->err.c_str() : "null group"; }

void lsq_dgroup_destroy(lsq_dgroup* g) {
    if (!g) return;
    for (int r = (int)g->h.size() - 1; r >= 0; --r) lsq_destroy(g->h[r]);
    delete g;
}

}  // extern "C"

// every rank's solve on its own host thread; the first failing rank's message is the group's
template <class F>
static int dgroup_run(lsq_dgroup* g, lsq_stats* s, F&& f) {
    if (!g || g->h.empty()) return -1;
    g->err.clear();
    const int n = (int)g->h.size();
    for (auto* h : g->h)
        if (!h->sys.dist) {
            g->err = "every rank of a device group needs lsq_dist_set_halo / lsq_dist_set_layout first";
            return -2;
        }
    std::vector<int> rc(n, 0);
    std::vector<lsq_stats> st(n);
    std::vector<std::thread> th;
    lsq::GroupFence fence(n);
    std::atomic<int> first_fail{-1};
    for (int r = 0; r < n; ++r)
        th.emplace_back([&, r] {
            std::memset(&st[r], 0, sizeof(lsq_stats));
            rc[r] = guarded(g->h[r], [&](lsq::System& S) {
                lsq::Group G;
                G.ranks = {&S};
                G.fence = &fence;
                return f(G, r, &st[r]);
            });
            // a failing rank releases the others from their next rendezvous (they fail too)
            if (rc[r] < 0 && fence.poison()) first_fail.store(r);
        });
    for (auto& t : th) t.join();
    if (first_fail.load() >= 0) {
        const int r = first_fail.load();
        g->err = "rank " + std::to_string(r) + ": " + g->h[r]->sys.err;
        return rc[r];
    }
    if (s) *s = st[0];
    return rc[0];
}

extern "C" {

int lsq_fence_selftest(int32_t n, int32_t fail_rank, int32_t rounds) {
    if (n < 1 || rounds < 1) return -1;
    lsq::GroupFence fence(n);
    std::atomic<int> left{0};
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
        th.emplace_back([&, r] {
            try {
                for (int k = 0; k < rounds; ++k) {
                    if (r == fail_rank && k == fail_rank % rounds) throw std::runtime_error("injected");
                    fence.arrive();
                }
            } catch (const lsq::GroupFence::Poisoned&) {
                left.fetch_add(1);
            } catch (const std::exception&) {
                fence.poison();
            }
        });
    for (auto& t : th) t.join();
    return left.load();
}

int lsq_dgroup_solve(lsq_dgroup* g, const double* const* b, double* const* x, const lsq_opts* o, lsq_stats* s) {
    if (!b || !x) return -1;
    lsq_opts d;
    lsq_default_opts(&d);
    const lsq_opts& oo = o ? *o : d;
    return dgroup_run(g, s, [&](lsq::Group& G, int r, lsq_stats* st) {
        double* xs[1] = {x[r]};
        return oo.method == 1 ? lsq::group_cg_solve(G, &b[r], xs, oo, st) : lsq::group_solve(G, &b[r], xs, oo, st);
    });
}

int lsq_dgroup_iterate(lsq_dgroup* g, const double* const* b, int64_t iters, const lsq_opts* o, lsq_stats* s) {
    if (!b) return -1;
    lsq_opts d;
    lsq_default_opts(&d);
    const lsq_opts& oo = o ? *o : d;
    return dgroup_run(g, s, [&](lsq::Group& G, int r, lsq_stats* st) {
        return oo.method == 1 ? lsq::group_cg_iterate(G, &b[r], iters, oo, st)
                              : lsq::group_iterate(G, &b[r], iters, oo, st);
    });
}

}  // extern "C"
