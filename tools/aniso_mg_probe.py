"""Probe: the anisotropic notebook system (z0-only 2-D lattice) on the structured path with the
multigrid preconditioner (precond 4, CGNR) against the band-preconditioned LSQR of
sparseqr_compat.solve.  Prints one JSON line per case."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from lssurf_amd import aniso, sparseqr_compat                  # noqa: E402
from lssurf_amd.smooth_fit import FitSystem                    # noqa: E402


def case(nodes, npts, band=True):
    G_data, Gc, E, rhs, g = aniso.system_ops(nodes=nodes, npts=npts)
    n = Gc.col_N
    out = dict(nodes=nodes, npts=npts, n=n)
    t0 = time.time()
    fs = FitSystem(G_data, Gc, np.arange(n), n)
    try:
        fs.solver.set_column_blocks_affine(n, [0], [1], [0], [1])
        fs.has_blocks = True
        out['form_s'] = time.time() - t0
        w = 1. / E
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.ones(w.size, bool))
        for pc in (4, 3):
            ok, why = fs.solver.cg_available(pc)
            out[f'cg{pc}_ok'] = bool(ok)
            if not ok:
                out[f'cg{pc}_why'] = why
                continue
            t0 = time.time()
            x, st = fs.solver.solve(rhs, precond=pc, method=1, atol=1e-12, btol=1e-12, conlim=1e12,
                                    maxit=200000)
            out[f'p{pc}'] = dict(s=time.time() - t0, iters=st['iters'], istop=st['istop'], time_s=st['time_s'],
                                 setup_s=st['setup_s'], method=st['method'])
            out[f'x{pc}'] = x
    finally:
        fs.close()
    if band:
        A, b, _ = aniso.system(nodes=nodes, npts=npts)
        t0 = time.time()
        xb = sparseqr_compat.solve(A, b)
        st = sparseqr_compat.solve.last_stats
        out['band'] = dict(s=time.time() - t0, iters=st['iters'], istop=st['istop'])
        for pc in (4, 3):
            if f'x{pc}' in out:
                x = out[f'x{pc}']
                out[f'p{pc}']['rel'] = float(np.linalg.norm(x - xb) / np.linalg.norm(xb))
                out[f'p{pc}']['maxabs'] = float(np.abs(x - xb).max())
    out.pop('x4', None)
    out.pop('x3', None)
    print(json.dumps(out, default=float), flush=True)


if __name__ == '__main__':
    for spec in sys.argv[1:]:
        nodes, npts = (int(v) for v in spec.split(':'))
        case(nodes, npts)
