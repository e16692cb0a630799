"""ctypes wrappers for the oracle's C restatements (TEST INFRASTRUCTURE ONLY).

build() compiles oracle/lsqr_cpu.c + oracle/cgnr_cpu.c + oracle/cgnr_struct_cpu.c + oracle/tri_upper.c into
oracle/_cpu.so with gcc -O2
-fopenmp (no -march: plain SSE2 doubles, no FMA — matching the reference's Cython build).
"""
import ctypes
import os
import subprocess

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, '_cpu.so')
SRC = [os.path.join(HERE, 'lsqr_cpu.c'), os.path.join(HERE, 'cgnr_cpu.c'), os.path.join(HERE, 'cgnr_struct_cpu.c'),
       os.path.join(HERE, 'tri_upper.c')]
_lib = None


def build(force=False):
    if not force and os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(s) for s in SRC):
        return LIB
    cmd = ['gcc', '-O2', '-fopenmp', '-fPIC', '-shared', '-ffp-contract=off', '-o', LIB, *SRC, '-lm']
    subprocess.run(cmd, check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        i64, i32, f64, f32 = ctypes.c_int64, ctypes.c_int32, ctypes.c_double, ctypes.c_float
        L.lsqr_cpu.argtypes = [i64, i64, P, P, P, P, P, f64, f64, f64, i64, ctypes.c_int, i64, ctypes.c_int, P]
        L.lsqr_cpu.restype = ctypes.c_int
        L.cgnr_bj_cpu.argtypes = [i64, i64, P, P, P, P, i64, P, P, P, f64, i64, i64, ctypes.c_int, P]
        L.cgnr_bj_cpu.restype = ctypes.c_int
        L.cgnr_bj_struct_cpu.argtypes = [i32, P, i32, P, i64, P, P, P, i32, P, i64, i64, P, i64, P, P, i64, P, P, P,
                                         f64, i64, i64, ctypes.c_int, P]
        L.cgnr_bj_struct_cpu.restype = ctypes.c_int
        L.oracle_inv_tr_upper.argtypes = [i64, P, P, P, i64, f32, P, P, P, P]
        L.oracle_inv_tr_upper.restype = ctypes.c_int
        L.oracle_propagate_qz_errors.argtypes = [i64, P, P, P, P]
        L.oracle_spsolve_tr_upper.argtypes = [i64, P, P, P, P, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _csr(A):
    A = sp.csr_matrix(A)
    rp = np.ascontiguousarray(A.indptr, dtype=np.int64)
    ci = np.ascontiguousarray(A.indices, dtype=np.int32)
    v = np.ascontiguousarray(A.data, dtype=np.float64)
    return A.shape, rp, ci, v


def lsqr(A, b, atol=1e-10, btol=1e-10, conlim=1e8, maxit=0, precond=1, fixed_iters=0, threads=0):
    """CPU LSQR on the final weighted A; returns (x, stats dict)."""
    (m, n), rp, ci, v = _csr(A)
    b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(n)
    st = np.zeros(10)
    lib().lsqr_cpu(m, n, _p(rp), _p(ci), _p(v), _p(b), _p(x), atol, btol, conlim, maxit, precond, fixed_iters,
                   threads, _p(st))
    keys = ['iters', 'istop', 'r1norm', 'r2norm', 'anorm', 'acond', 'arnorm', 'xnorm', 'time_s', 'threads']
    return x, dict(zip(keys, st.tolist()))


def cgnr_bj(A, b, block_ptr, block_cols, atol=1e-10, maxit=0, fixed_iters=0, threads=0):
    """CPU CGNR + block-Jacobi (oracle/cgnr_cpu.c) on the final weighted A with the GPU solve's
    column blocks (compact ids); returns (x, stats dict)."""
    (m, n), rp, ci, v = _csr(A)
    b = np.ascontiguousarray(b, dtype=np.float64)
    bp = np.ascontiguousarray(block_ptr, dtype=np.int64)
    bc = np.ascontiguousarray(block_cols, dtype=np.int32)
    x = np.zeros(n)
    st = np.zeros(7)
    rc = lib().cgnr_bj_cpu(m, n, _p(rp), _p(ci), _p(v), _p(b), bp.size - 1, _p(bp), _p(bc), _p(x), atol, maxit,
                           fixed_iters, threads, _p(st))
    if rc != 0:
        raise ValueError('cgnr_bj: a block has more than 16 columns')
    keys = ['iters', 'time_s', 'setup_s', 'threads', 'snorm', 'rnorm', 'anorm_f']
    return x, dict(zip(keys, st.tolist()))


def cgnr_bj_struct(desc, n_full, row_scale, keep_cols, b, block_ptr, block_cols, atol=1e-10, maxit=0,
                   fixed_iters=0, threads=0):
    """CPU CGNR + block-Jacobi on the STRUCTURED operator (oracle/cgnr_struct_cpu.c: stencil rows from
    the part descriptors, matrix-free data rows from the sorted points — the GPU line's operator
    representation, no stored matrix).  desc: lssurf_amd.assemble.describe(G_data, Gc) (grids,
    interp grid ids, (py, px, pt), stencils, npts); row_scale: row weights × mask (m); keep_cols:
    compact -> full column ids; b: the weighted rhs (m).  Returns (x, stats) as cgnr_bj; raises
    ValueError when the interpolation grids do not share one (y, x) lattice."""
    grids, interp, (py, px, pt), stencils, npts = desc[:5]
    if len(desc) > 5 and desc[5]:
        raise ValueError('cgnr_bj_struct: field-valued stencil parts are not supported')
    ga = (type(grids[0]) * len(grids))(*grids)
    sa = (type(stencils[0]) * len(stencils))(*stencils)
    ig = np.ascontiguousarray(interp, dtype=np.int32)
    rs = np.ascontiguousarray(row_scale, dtype=np.float64)
    kc = np.ascontiguousarray(keep_cols, dtype=np.int64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    bp = np.ascontiguousarray(block_ptr, dtype=np.int64)
    bc = np.ascontiguousarray(block_cols, dtype=np.int32)
    py, px = np.ascontiguousarray(py, np.float64), np.ascontiguousarray(px, np.float64)
    ptv = None if pt is None else np.ascontiguousarray(pt, np.float64)
    x = np.zeros(kc.size)
    st = np.zeros(7)
    rc = lib().cgnr_bj_struct_cpu(len(grids), ctypes.cast(ga, ctypes.c_void_p), ig.size, _p(ig), int(npts), _p(py),
                                  _p(px), None if ptv is None else _p(ptv), len(stencils),
                                  ctypes.cast(sa, ctypes.c_void_p), rs.size, int(n_full), _p(rs), kc.size, _p(kc),
                                  _p(b), bp.size - 1, _p(bp), _p(bc), _p(x), atol, maxit, fixed_iters, threads, _p(st))
    if rc == -2:
        raise ValueError('cgnr_bj_struct: the interpolation grids do not share one (y, x) lattice')
    if rc != 0:
        raise ValueError('cgnr_bj_struct: a block has more than 16 columns')
    keys = ['iters', 'time_s', 'setup_s', 'threads', 'snorm', 'rnorm', 'anorm_f']
    return x, dict(zip(keys, st.tolist()))


def inv_tr_upper(R, nnz, tol):
    (N, _), rp, ci, v = _csr(R)
    rp = rp.astype(np.int32)
    rr = np.zeros(nnz, np.int32)
    cc = np.zeros(nnz, np.int32)
    vv = np.zeros(nnz)
    n_out = np.zeros(1, np.int64)
    st = lib().oracle_inv_tr_upper(N, _p(rp), _p(ci), _p(v), nnz, tol, _p(rr), _p(cc), _p(vv), _p(n_out))
    k = int(n_out[0])
    return rr[:k], cc[:k], vv[:k], st


def propagate_qz_errors(R):
    (N, _), rp, ci, v = _csr(R)
    rp = rp.astype(np.int32)
    E = np.zeros(N)
    lib().oracle_propagate_qz_errors(N, _p(rp), _p(ci), _p(v), _p(E))
    return E


def spsolve_tr_upper(R, b):
    (N, _), rp, ci, v = _csr(R)
    rp = rp.astype(np.int32)
    b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(N)
    lib().oracle_spsolve_tr_upper(N, _p(rp), _p(ci), _p(v), _p(b), _p(x))
    return x
