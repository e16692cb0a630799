"""Development: the multigrid solve over N virtual ranks on one GPU (every rank's kernels on one
stream, exchanges as device copies): iterations, solve time (the SUM of the ranks' work — a proxy
for the per-rank cost when divided by N), set-up, and the bytes one rank would send per iteration.
LSQ_MG_PART=0 replicates every coarse level (round-3 design) for the A/B.

    python tools/vgroup_bench.py c4 4"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(config, nranks):
    import lssurf_amd as LS
    from lssurf_amd import dist, synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    D, kw = synthetic.points(config)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    w = 1. / np.concatenate((S['Ed'], S['Ec']))
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    t0 = time.time()
    vd = dist.VirtualDistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, nranks)
    form = time.time() - t0
    out = {'config': config, 'nranks': nranks, 'part': os.environ.get('LSQ_MG_PART', '1'), 'formation_s': form}
    try:
        for label in ('first', 'timed'):
            t0 = time.time()
            x = vd.solve(w if label == 'first' else None, rhs, atol=1e-10, btol=1e-10, conlim=1e8, precond=4, method=1)
            st = dict(vd.stats)
            out[label] = {'wall_s': time.time() - t0, 'iters': int(st['iters']), 'istop': int(st['istop']),
                          'time_s': st['time_s'], 'comm_bytes_per_iter': st['comm_bytes_per_iter']}
        out['x_norm'] = float(np.linalg.norm(x))
    finally:
        vd.close()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]))
