/* lsqr_cpu.c — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
 *
 * C/OpenMP restatement of Paige & Saunders' LSQR exactly as scipy.sparse.linalg.lsqr states it
 * (scipy 1.15 _isolve/lsqr.py: recurrences, _sym_ortho, stopping tests istop 1..7), operating
 * on a CSR matrix A (int64 row pointers, int32 columns, f64 values) and its explicit
 * transpose.  Optional right preconditioning by column scaling (x = D y, D = 1/||A_:,j||),
 * the same preconditioner liblsqsurf applies, so iteration counts are comparable.
 *
 * Role: (1) parity checker for lssurf_amd's LSQR at sizes the dense oracle cannot reach;
 *       (2) bench.py's cpu_baseline ("port": the reference's CPU path is SuiteSparseQR, absent).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static double now_s(void) { return omp_get_wtime(); }

static void spmv(int64_t m, const int64_t* rp, const int32_t* ci, const double* v, const double* x, double* y) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < m; ++i) {
        double a = 0.0;
        for (int64_t e = rp[i]; e < rp[i + 1]; ++e) a += v[e] * x[ci[e]];
        y[i] = a;
    }
}

static double nrm2(int64_t n, const double* x) {
    double s = 0.0;
#pragma omp parallel for reduction(+ : s) schedule(static)
    for (int64_t i = 0; i < n; ++i) s += x[i] * x[i];
    return sqrt(s);
}

static double sgn(double x) { return x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0); }

static void sym_ortho(double a, double b, double* c, double* s, double* r) {
    if (b == 0.0) { *c = sgn(a); *s = 0.0; *r = fabs(a); return; }
    if (a == 0.0) { *c = 0.0; *s = sgn(b); *r = fabs(b); return; }
    if (fabs(b) > fabs(a)) {
        double tau = a / b;
        *s = sgn(b) / sqrt(1 + tau * tau);
        *c = *s * tau;
        *r = b / *s;
    } else {
        double tau = b / a;
        *c = sgn(a) / sqrt(1 + tau * tau);
        *s = *c * tau;
        *r = a / *c;
    }
}

/* CSR transpose (deterministic, serial scatter in row order). */
static void transpose(int64_t m, int64_t n, const int64_t* rp, const int32_t* ci, const double* v,
                      int64_t* trp, int32_t* tci, double* tv) {
    memset(trp, 0, sizeof(int64_t) * (n + 1));
    for (int64_t e = 0; e < rp[m]; ++e) trp[ci[e] + 1]++;
    for (int64_t j = 0; j < n; ++j) trp[j + 1] += trp[j];
    int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
    memcpy(cur, trp, sizeof(int64_t) * n);
    for (int64_t i = 0; i < m; ++i)
        for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
            int64_t p = cur[ci[e]]++;
            tci[p] = (int32_t)i;
            tv[p] = v[e];
        }
    free(cur);
}

/* stats: [iters, istop, r1norm, r2norm, anorm, acond, arnorm, xnorm, time_s, threads]
 * fixed_iters > 0: run exactly that many iterations (timing sample), no stopping test. */
int lsqr_cpu(int64_t m, int64_t n, const int64_t* rp, const int32_t* ci, const double* val, const double* b,
             double* x, double atol, double btol, double conlim, int64_t maxit, int precond, int64_t fixed_iters,
             int nthreads, double* stats) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
    const int64_t nnz = rp[m];
    double* av = (double*)malloc(sizeof(double) * (nnz > 0 ? nnz : 1));
    int64_t* trp = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int32_t* tci = (int32_t*)malloc(sizeof(int32_t) * (nnz > 0 ? nnz : 1));
    double* tv = (double*)malloc(sizeof(double) * (nnz > 0 ? nnz : 1));
    double* d = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
    double *u = (double*)malloc(sizeof(double) * m), *v = (double*)malloc(sizeof(double) * n);
    double *w = (double*)malloc(sizeof(double) * n), *t = (double*)malloc(sizeof(double) * (m > n ? m : n));
    double* y = (double*)calloc(n, sizeof(double));
    memcpy(av, val, sizeof(double) * nnz);
    transpose(m, n, rp, ci, av, trp, tci, tv);
    for (int64_t j = 0; j < n; ++j) {
        double s = 0.0;
        for (int64_t e = trp[j]; e < trp[j + 1]; ++e) s += tv[e] * tv[e];
        d[j] = (precond == 1 && s > 0.0) ? 1.0 / sqrt(s) : 1.0;
    }
    if (precond == 1) {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < m; ++i)
            for (int64_t e = rp[i]; e < rp[i + 1]; ++e) av[e] *= d[ci[e]];
#pragma omp parallel for schedule(static)
        for (int64_t j = 0; j < n; ++j)
            for (int64_t e = trp[j]; e < trp[j + 1]; ++e) tv[e] *= d[j];
    }
    const double eps = 2.220446049250313e-16;
    if (maxit <= 0) maxit = 4 * n;
    const double ctol = conlim > 0 ? 1.0 / conlim : 0.0;
    double anorm = 0, acond = 0, ddnorm = 0, res2 = 0, xnorm = 0, xxnorm = 0, z = 0, cs2 = -1, sn2 = 0;
    memcpy(u, b, sizeof(double) * m);
    double bnorm = nrm2(m, u), beta = bnorm, alfa = 0;
    if (beta > 0) {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < m; ++i) u[i] /= beta;
        spmv(n, trp, tci, tv, u, v);
        alfa = nrm2(n, v);
    } else {
        memset(v, 0, sizeof(double) * n);
    }
    if (alfa > 0) {
#pragma omp parallel for schedule(static)
        for (int64_t j = 0; j < n; ++j) v[j] /= alfa;
    }
    memcpy(w, v, sizeof(double) * n);
    double rhobar = alfa, phibar = beta, rnorm = beta, r1norm = beta, r2norm = beta, arnorm = alfa * beta;
    int64_t itn = 0;
    int istop = 0;
    double t0 = now_s();
    if (arnorm != 0) {
        while (itn < maxit) {
            itn++;
            spmv(m, rp, ci, av, v, t);
#pragma omp parallel for schedule(static)
            for (int64_t i = 0; i < m; ++i) u[i] = t[i] - alfa * u[i];
            beta = nrm2(m, u);
            if (beta > 0) {
#pragma omp parallel for schedule(static)
                for (int64_t i = 0; i < m; ++i) u[i] /= beta;
                anorm = sqrt(anorm * anorm + alfa * alfa + beta * beta);
                spmv(n, trp, tci, tv, u, t);
#pragma omp parallel for schedule(static)
                for (int64_t j = 0; j < n; ++j) v[j] = t[j] - beta * v[j];
                alfa = nrm2(n, v);
                if (alfa > 0) {
#pragma omp parallel for schedule(static)
                    for (int64_t j = 0; j < n; ++j) v[j] /= alfa;
                }
            }
            double cs, sn, rho;
            sym_ortho(rhobar, beta, &cs, &sn, &rho);
            double theta = sn * alfa;
            rhobar = -cs * alfa;
            double phi = cs * phibar;
            phibar = sn * phibar;
            double tau = sn * phi;
            double t1 = phi / rho, t2 = -theta / rho;
            double wn = 0.0;
#pragma omp parallel for reduction(+ : wn) schedule(static)
            for (int64_t j = 0; j < n; ++j) {
                double wj = w[j];
                wn += wj * wj;
                y[j] += t1 * wj;
                w[j] = v[j] + t2 * wj;
            }
            ddnorm += wn / (rho * rho);
            double delta = sn2 * rho, gambar = -cs2 * rho, rhs = phi - delta * z;
            double zbar = rhs / gambar;
            xnorm = sqrt(xxnorm + zbar * zbar);
            double gamma = sqrt(gambar * gambar + theta * theta);
            cs2 = gambar / gamma;
            sn2 = theta / gamma;
            z = rhs / gamma;
            xxnorm += z * z;
            acond = anorm * sqrt(ddnorm);
            double res1 = phibar * phibar;
            rnorm = sqrt(res1 + res2);
            arnorm = alfa * fabs(tau);
            r1norm = rnorm;
            r2norm = rnorm;
            if (fixed_iters > 0) {
                if (itn >= fixed_iters) { istop = 7; break; }
                continue;
            }
            double test1 = rnorm / bnorm, test2 = arnorm / (anorm * rnorm + eps), test3 = 1 / (acond + eps);
            double tt1 = test1 / (1 + anorm * xnorm / bnorm);
            double rtol = btol + atol * anorm * xnorm / bnorm;
            if (itn >= maxit) istop = 7;
            if (1 + test3 <= 1) istop = 6;
            if (1 + test2 <= 1) istop = 5;
            if (1 + tt1 <= 1) istop = 4;
            if (test3 <= ctol) istop = 3;
            if (test2 <= atol) istop = 2;
            if (test1 <= rtol) istop = 1;
            if (istop) break;
        }
    }
    double t1s = now_s();
    for (int64_t j = 0; j < n; ++j) x[j] = d[j] * y[j];
    if (stats) {
        stats[0] = (double)itn; stats[1] = istop; stats[2] = r1norm; stats[3] = r2norm; stats[4] = anorm;
        stats[5] = acond; stats[6] = arnorm; stats[7] = xnorm; stats[8] = t1s - t0;
        stats[9] = (double)omp_get_max_threads();
    }
    free(av); free(trp); free(tci); free(tv); free(d); free(u); free(v); free(w); free(t); free(y);
    return istop;
}
