"""ctypes binding of liblsqsurf.so (include/lsqsurf.h).  Product path: there is no fallback —
if the library is missing or no gfx950 device is present, every call raises."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'liblsqsurf.so')


class NativeError(RuntimeError):
    pass


class NativeRefused(NativeError):
    """Status -5: declined for lack of resources (include/lsqsurf.h); another method may run."""
    pass


class LsqOpts(ctypes.Structure):
    _fields_ = [('method', ctypes.c_int32), ('precond', ctypes.c_int32), ('atol', ctypes.c_double),
                ('btol', ctypes.c_double), ('conlim', ctypes.c_double), ('maxit', ctypes.c_int64),
                ('use_x0', ctypes.c_int32), ('batch', ctypes.c_int32), ('use_graph', ctypes.c_int32),
                ('op', ctypes.c_int32), ('b_rows', ctypes.c_int64),
                ('anorm0', ctypes.c_double)]


class GridDesc(ctypes.Structure):
    _fields_ = [('ndim', ctypes.c_int32), ('reserved', ctypes.c_int32), ('shape', ctypes.c_int64 * 3),
                ('col0', ctypes.c_int64), ('b0', ctypes.c_double * 3), ('delta', ctypes.c_double * 3)]


class StencilDesc(ctypes.Structure):
    _fields_ = [('grid', ctypes.c_int32), ('ntpl', ctypes.c_int32), ('off', (ctypes.c_int32 * 3) * 8),
                ('val', ctypes.c_double * 8), ('row0', ctypes.c_int64), ('n_eq', ctypes.c_int64),
                ('lo', ctypes.c_int64 * 3), ('hi', ctypes.c_int64 * 3)]


class LsqStats(ctypes.Structure):
    _fields_ = [('iters', ctypes.c_int64), ('istop', ctypes.c_int32), ('method', ctypes.c_int32),
                ('r1norm', ctypes.c_double), ('r2norm', ctypes.c_double), ('anorm', ctypes.c_double),
                ('acond', ctypes.c_double), ('arnorm', ctypes.c_double), ('xnorm', ctypes.c_double),
                ('time_s', ctypes.c_double), ('bytes_per_iter', ctypes.c_double), ('setup_s', ctypes.c_double),
                ('comm_bytes_per_iter', ctypes.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


# every symbol declared in include/lsqsurf.h
EXPORTS = ['lsq_default_opts', 'lsq_create', 'lsq_destroy', 'lsq_last_error', 'lsq_set_col_map',
           'lsq_set_matrix_coo', 'lsq_set_matrix_stencil', 'lsq_set_stencil_fields', 'lsq_set_row_weight',
           'lsq_set_row_mask',
           'lsq_set_column_blocks', 'lsq_set_column_blocks_affine', 'lsq_shape', 'lsq_get_csr', 'lsq_release_full_csr',
           'lsq_solve', 'lsq_spmv', 'lsq_spmv_rows', 'lsq_rows_sumsq', 'lsq_data_colsum', 'lsq_iterate', 'lsq_profile_kernels', 'lsq_cg_available', 'lsq_profile_cg', 'lsq_mg_info', 'lsq_mg_apply', 'lsq_normal_apply', 'lsq_sell_info', 'lsq_sigma_x', 'lsq_cov_band', 'lsq_cov_band_window', 'lsq_cov_band_windows', 'lsq_cov_band_windows_schur', 'lsq_set_band_order', 'lsq_band_factor',
           'lsq_get_rinv', 'lsq_dist_unique_id', 'lsq_create_dist', 'lsq_dist_comm_info', 'lsq_dist_referenced_cols',
           'lsq_dist_set_layout', 'lsq_dist_set_halo', 'lsq_dist_set_global', 'lsq_vgroup_create', 'lsq_vgroup_rank', 'lsq_vgroup_solve', 'lsq_vgroup_iterate',
           'lsq_vgroup_last_error', 'lsq_vgroup_destroy',
           'lsq_dgroup_create', 'lsq_dgroup_rank', 'lsq_dgroup_solve', 'lsq_dgroup_iterate', 'lsq_dgroup_last_error',
           'lsq_dgroup_destroy', 'lsq_fence_selftest',
           'lsq_rde_create', 'lsq_rde_order_stats', 'lsq_rde_last_error', 'lsq_rde_destroy',
           'tri_upper_solve_csr', 'tri_upper_inv_csr', 'tri_upper_rowrss_csr', 'tri_last_error']

_lib = None


def load():
    """Load liblsqsurf.so (in-tree build).  Raises NativeError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(f'{LIB_PATH} not built: run `python -m lssurf_amd.build` (hipcc, gfx950)')
    L = ctypes.CDLL(LIB_PATH)
    P, i32, i64, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    sig = {
        'lsq_default_opts': ([P], None),
        'lsq_create': ([i32], P),
        'lsq_destroy': ([P], None),
        'lsq_last_error': ([P], ctypes.c_char_p),
        'lsq_set_col_map': ([P, i64, P, i64], ctypes.c_int),
        'lsq_set_matrix_coo': ([P, i64, i64, i64, P, P, P, P], ctypes.c_int),
        'lsq_set_row_weight': ([P, P], ctypes.c_int),
        'lsq_set_matrix_stencil': ([P, i64, i64, i32, P, i32, P, i64, P, P, P, i32, P, P], ctypes.c_int),
        'lsq_set_stencil_fields': ([P, i32, i32, P, P, i32, P, i64, P], ctypes.c_int),
        'lsq_set_row_mask': ([P, P], ctypes.c_int),
        'lsq_set_column_blocks': ([P, i64, P, P], ctypes.c_int),
        'lsq_set_column_blocks_affine': ([P, i64, i32, P, P, P, P], ctypes.c_int),
        'lsq_shape': ([P, P, P, P], ctypes.c_int),
        'lsq_get_csr': ([P, P, P, P], ctypes.c_int),
        'lsq_release_full_csr': ([P, P], ctypes.c_int),
        'lsq_solve': ([P, P, P, P, P], ctypes.c_int),
        'lsq_spmv': ([P, i32, P, P], ctypes.c_int),
        'lsq_spmv_rows': ([P, i64, i64, P, P], ctypes.c_int),
        'lsq_rows_sumsq': ([P, P, i32, P, P, P, P], ctypes.c_int),
        'lsq_data_colsum': ([P, P, P], ctypes.c_int),
        'lsq_iterate': ([P, P, i64, P, P], ctypes.c_int),
        'lsq_profile_kernels': ([P, i32, i32, P], ctypes.c_int),
        'lsq_cg_available': ([P, i32], ctypes.c_int),
        'lsq_profile_cg': ([P, i32, i32, P], ctypes.c_int),
        'lsq_mg_info': ([P, P, i64], ctypes.c_int),
        'lsq_mg_apply': ([P, i32, i32, P, P], ctypes.c_int),
        'lsq_normal_apply': ([P, P, P], ctypes.c_int),
        'lsq_sell_info': ([P, P], ctypes.c_int),
        'lsq_sigma_x': ([P, P], ctypes.c_int),
        'lsq_get_rinv': ([P, P], ctypes.c_int),
        'lsq_cov_band': ([P, P, P, ctypes.c_int64, P, P, P, P, P], ctypes.c_int),
        'lsq_cov_band_window': ([P, P, i64, P, P, i64, P, P, P, P, P], ctypes.c_int),
        'lsq_cov_band_windows': ([P, i64, P, P, P, P, P, P, P, P, P, P], ctypes.c_int),
        'lsq_cov_band_windows_schur': ([P, i64, P, P, P, P, P, P, P, P], ctypes.c_int),
        'lsq_set_band_order': ([P, ctypes.c_int64, P], ctypes.c_int),
        'lsq_band_factor': ([P, P, P, P, P, P], ctypes.c_int),
        'lsq_dist_unique_id': ([P], ctypes.c_int),
        'lsq_create_dist': ([i32, i32, i32, P], P),
        'lsq_dist_comm_info': ([P, P], ctypes.c_int),
        'lsq_dist_referenced_cols': ([P, P], ctypes.c_int),
        'lsq_dist_set_layout': ([P, P, i64, i64, i32, P, P, P, P], ctypes.c_int),
        'lsq_dist_set_halo': ([P, i32, P, i32, P, P, P, P, P], ctypes.c_int),
        'lsq_dist_set_global': ([P, i64, i32, P, i32, P, P, i32, i32, i32, i32], ctypes.c_int),
        'lsq_vgroup_create': ([i32, i32], P),
        'lsq_vgroup_rank': ([P, i32], P),
        'lsq_vgroup_solve': ([P, P, P, P, P], ctypes.c_int),
        'lsq_vgroup_iterate': ([P, P, i64, P, P], ctypes.c_int),
        'lsq_vgroup_last_error': ([P], ctypes.c_char_p),
        'lsq_vgroup_destroy': ([P], None),
        'lsq_dgroup_create': ([i32, P], P),
        'lsq_dgroup_rank': ([P, i32], P),
        'lsq_dgroup_solve': ([P, P, P, P, P], ctypes.c_int),
        'lsq_dgroup_iterate': ([P, P, i64, P, P], ctypes.c_int),
        'lsq_dgroup_last_error': ([P], ctypes.c_char_p),
        'lsq_dgroup_destroy': ([P], None),
        'lsq_fence_selftest': ([ctypes.c_int32, ctypes.c_int32, ctypes.c_int32], ctypes.c_int),
        'lsq_rde_create': ([i32, i64, P, P], P),
        'lsq_rde_order_stats': ([P, f64, i64, P, P], ctypes.c_int),
        'lsq_rde_last_error': ([P], ctypes.c_char_p),
        'lsq_rde_destroy': ([P], None),
        'tri_upper_solve_csr': ([i32, i64, P, P, P, P, P], ctypes.c_int),
        'tri_upper_inv_csr': ([i32, i64, P, P, P, i64, ctypes.c_float, P, P, P, P], ctypes.c_int),
        'tri_upper_rowrss_csr': ([i32, i64, P, P, P, P], ctypes.c_int),
        'tri_last_error': ([], ctypes.c_char_p),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def as_c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def default_opts(**kw):
    o = LsqOpts()
    load().lsq_default_opts(ctypes.byref(o))
    for k, v in kw.items():
        if v is not None:
            setattr(o, k, v)
    return o
