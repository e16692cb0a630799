"""lssurf_amd — MI355X-native least-squares solve path of SmithB/LSsurf.

Drop-in names (LSsurf/__init__.py): fd_grid, lin_op, smooth_fit, iterate_fit, RDE,
setup_smoothness_constraints, build_reference_epoch_matrix, setup_grids, calc_sigma_extra,
inv_tr_upper / propagate_qz_errors / spsolve_tr_upper (GPU kernels behind the same
signatures).  The solve runs in liblsqsurf.so (HIP, gfx950); see DESIGN.md.
"""
from .fd_grid import fd_grid
from .lin_op import lin_op
from .calc_sigma_extra import RDE, calc_sigma_extra, calc_sigma_extra_on_grid
from .constraint_functions import setup_smoothness_constraints, build_reference_epoch_matrix
from .grid_functions import setup_grids, sum_cell_area, calc_cell_area, setup_averaging_ops, validate_by_dz_mask
from .solver import LSQSolver, inv_tr_upper, propagate_qz_errors, spsolve_tr_upper
from .smooth_fit import smooth_fit, iterate_fit, parse_model, FitSystem
from . import containers

__all__ = ['fd_grid', 'lin_op', 'RDE', 'calc_sigma_extra', 'calc_sigma_extra_on_grid',
           'setup_smoothness_constraints', 'build_reference_epoch_matrix', 'setup_grids', 'sum_cell_area',
           'calc_cell_area', 'setup_averaging_ops', 'validate_by_dz_mask', 'LSQSolver', 'inv_tr_upper',
           'propagate_qz_errors', 'spsolve_tr_upper', 'smooth_fit', 'iterate_fit', 'parse_model', 'FitSystem',
           'containers']
