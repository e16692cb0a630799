"""Development: a short multigrid CGNR solve at a BASELINE config (maxit iterations), the program the
PMC passes of tools/gpu_r4l.sh count.  Usage: python tools/mg_pmc_probe.py [config] [maxit]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(cfg, maxit):
    import lssurf_amd as LS
    from lssurf_amd import synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    from lssurf_amd.smooth_fit import FitSystem
    D, kw = synthetic.points(cfg)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    w = 1. / np.concatenate((S['Ed'], S['Ec']))
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    try:
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.ones(w.size, bool))
        x, st = fs.solver.solve(rhs, atol=1e-14, btol=1e-14, maxit=maxit, precond=4, method=1)
        print('iters', st['iters'], flush=True)
    finally:
        fs.close()


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'c4', int(sys.argv[2]) if len(sys.argv) > 2 else 6)
