"""Development: the convergence curve of the multigrid CGNR solve at C5a (the anisotropic config)
around smooth_fit's stopping rule — the rule's ratio ‖Aᵀr‖ / (‖A‖‖r‖) (stats arnorm, anorm, rnorm)
after k iterations for a range of k, and the iteration count at several atol.  Answers whether the
61 → 72 iteration change between two builds is a plateau of the ratio near atol = 1e-10 (a rounding-
level perturbation moves the stop) or a weaker preconditioner.

    python tools/c5a_conv.py [config [seed id]]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(cfg, seed=None):
    from lssurf_amd import synthetic
    from lssurf_amd.smooth_fit import FitSystem
    S, _ = synthetic.aniso_system(cfg) if seed is None else synthetic.aniso_system(cfg, config_id=seed)
    fs = FitSystem(S['G_data'], S['Gc'], S['keep'], S['Gc'].col_N, grids=S['grids'])
    try:
        fs.solver.set_row_weight(S['w'])
        fs.solver.set_row_mask(np.ones(S['w'].size, bool))
        for precond in (4, 3):
            for atol in (1e-9, 3e-10, 1e-10, 3e-11):
                x, st = fs.solver.solve(S['rhs'], atol=atol, btol=atol, conlim=1e8, precond=precond, method=1)
                print(json.dumps({'precond': precond, 'atol': atol, 'iters': int(st['iters']), 'istop': int(st['istop']),
                                  'ratio': float(st['arnorm'] / (st['anorm'] * st['r2norm']))}), flush=True)
        for k in (30, 40, 50, 55, 60, 65, 70, 75, 80):
            x, st = fs.solver.solve(S['rhs'], atol=1e-14, btol=1e-14, conlim=1e8, maxit=k, precond=4, method=1)
            print(json.dumps({'precond': 4, 'maxit': k, 'iters': int(st['iters']),
                              'ratio': float(st['arnorm'] / (st['anorm'] * st['r2norm'])),
                              'anorm': float(st['anorm']), 'r2norm': float(st['r2norm']), 'arnorm': float(st['arnorm'])}),
                  flush=True)
    finally:
        fs.close()


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'c5a', int(sys.argv[2]) if len(sys.argv) > 2 else None)
