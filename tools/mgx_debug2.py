"""Development probe: the test's call order (hierarchy built at default weights, then a solve at
the system's weights) on a golden system."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from test_gpu_cgnr import _golden_system, TOL
for name in sys.argv[1:]:
    for variant in ('avail-first', 'weights-first', 'twice'):
        g, fs, w, rhs = _golden_system(name)
        if variant == 'weights-first':
            fs.solver.set_row_weight(w)
        if variant != 'twice':
            print(name, variant, 'cg4', fs.solver.cg_available(4))
        xm = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=4, method=1, maxit=5000, **TOL)
        if variant == 'twice':
            xm = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=4, method=1, maxit=5000, **TOL)
        print(name, variant, 'iters', fs.stats['iters'], fs.stats['istop'], 'rel err',
              np.linalg.norm(xm - g['x']) / np.linalg.norm(g['x']), flush=True)
        fs.close()
