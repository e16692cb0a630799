"""Timing of sparseqr_compat.solve on the anisotropic notebook system (BASELINE C5's constraint)
at growing sizes: band-preconditioned LSQR (precond 5) vs column-scaled LSQR (capped).

    python tools/bench_aniso.py 401:0 1025:2000000 2048:8000000     # nodes:points
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from lssurf_amd import aniso  # noqa: E402
from lssurf_amd import sparseqr_compat as sparseqr  # noqa: E402
from lssurf_amd.solver import LSQSolver  # noqa: E402


def main(specs, cap=2000):
    for spec in specs:
        nodes, npts = (int(v) for v in spec.split(':'))
        t0 = time.time()
        A, b, g = aniso.system(nodes, npts=npts)
        rec = {'nodes': nodes, 'points': npts, 'n': int(A.shape[1]), 'm': int(A.shape[0]), 'nnz': int(A.nnz),
               'host_build_s': time.time() - t0}
        perm, bw = sparseqr.band_order(A)
        rec['ata_half_bandwidth'] = bw
        with LSQSolver(0) as s:
            t0 = time.time()
            s.set_matrix_coo(A.shape[0], A.shape[1], A.row, A.col, A.data)
            rec['device_formation_s'] = time.time() - t0
            t0 = time.time()
            x, st = s.solve(b, atol=1e-12, btol=1e-12, conlim=1e12, precond=5)
            rec.update(band_solve_s=time.time() - t0, band_iters=st['iters'], band_istop=st['istop'],
                       band_device_s=st['time_s'])
            t0 = time.time()
            x1, st1 = s.solve(b, atol=1e-12, btol=1e-12, conlim=1e12, precond=1, maxit=cap)
            rec.update(colscale_s_capped=time.time() - t0, colscale_iters=st1['iters'], colscale_istop=st1['istop'],
                       colscale_rel_diff=float(np.linalg.norm(x1 - x) / np.linalg.norm(x)))
        print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main(sys.argv[1:] or ['401:0'])
