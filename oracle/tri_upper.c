/* tri_upper.c — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
 *
 * Plain-C restatement of the reference's Cython triangular kernels (compiled without FMA, like
 * the Cython build on x86-64):
 *   inv_tr_upper         LSsurf/inv_tr_upper.pyx:19-94
 *   propagate_qz_errors  LSsurf/propagate_qz_errors.pyx:15-69
 *   spsolve_tr_upper     LSsurf/spsolve_tr_upper.pyx:11-54
 * R is upper-triangular CSR with sorted int32 indices and the diagonal first in each row.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* column-by-column back substitution of R X = I, restricted to columns <= col (the .pyx
 * breaks at the first index > col); emit (i, col, x) when i == col or |x| > tol.
 * Returns status (1 when the output buffer of nnz entries is full), *n_out = entries. */
int oracle_inv_tr_upper(int64_t N, const int32_t* indptr, const int32_t* indices, const double* data, int64_t nnz,
                        float tol, int32_t* out_rows, int32_t* out_cols, double* out_vals, int64_t* n_out) {
    double* x = (double*)malloc(sizeof(double) * (N > 0 ? N : 1));
    int64_t out_ind = -1, max_ind = nnz - 1;
    int status = 0;
    memset(out_rows, 0, sizeof(int32_t) * nnz);
    memset(out_cols, 0, sizeof(int32_t) * nnz);
    memset(out_vals, 0, sizeof(double) * nnz);
    for (int64_t col = N - 1; col >= 0 && !status; --col) {
        memset(x, 0, sizeof(double) * N);
        x[col] = 1.0;
        for (int64_t i = col; i >= 0; --i) {
            double v = x[i];
            for (int64_t k = indptr[i] + 1; k < indptr[i + 1]; ++k) {
                if (indices[k] > col) break;
                v -= data[k] * x[indices[k]];
            }
            v /= data[indptr[i]];
            x[i] = v;
            if (i == col || fabs(v) > (double)tol) {
                out_ind += 1;
                if (out_ind >= max_ind) { status = 1; break; }
                out_rows[out_ind] = (int32_t)i;
                out_cols[out_ind] = (int32_t)col;
                out_vals[out_ind] = v;
            }
        }
    }
    *n_out = out_ind + 1;
    free(x);
    return status;
}

void oracle_propagate_qz_errors(int64_t N, const int32_t* indptr, const int32_t* indices, const double* data,
                                double* E) {
    double* x = (double*)malloc(sizeof(double) * (N > 0 ? N : 1));
    memset(E, 0, sizeof(double) * N);
    for (int64_t col = N - 1; col >= 0; --col) {
        memset(x, 0, sizeof(double) * N);
        x[col] = 1.0;
        for (int64_t i = col; i >= 0; --i) {
            double v = x[i];
            for (int64_t k = indptr[i] + 1; k < indptr[i + 1]; ++k) {
                if (indices[k] > col) break;
                v -= data[k] * x[indices[k]];
            }
            v /= data[indptr[i]];
            x[i] = v;
            E[i] += v * v;
        }
    }
    for (int64_t i = 0; i < N; ++i) E[i] = sqrt(E[i]);
    free(x);
}

void oracle_spsolve_tr_upper(int64_t N, const int32_t* indptr, const int32_t* indices, const double* data,
                             const double* b, double* x) {
    memcpy(x, b, sizeof(double) * N);
    for (int64_t i = N - 1; i >= 0; --i) {
        double v = x[i];
        for (int64_t k = indptr[i] + 1; k < indptr[i + 1]; ++k) v -= data[k] * x[indices[k]];
        v /= data[indptr[i]];
        x[i] = v;
    }
}
