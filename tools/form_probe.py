"""Development probe: device formation of a BASELINE config (FitSystem: upload, row generation,
transposes, SELL / dmf builds) timed from Python; run under rocprofv3 --kernel-trace --stats for
the per-kernel split.  Usage: python tools/form_probe.py [config]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(cfg, reps=1):
    import lssurf_amd as LS
    from lssurf_amd import synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    D, kw = synthetic.points(cfg)
    t0 = time.time()
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    t1 = time.time()
    from lssurf_amd.solver import LSQSolver
    from lssurf_amd.assemble import describe
    from lssurf_amd.constraint_functions import node_column_blocks
    G_data, Gc, n_full = S['G_data'], S['Gc'], S['Gc'].col_N
    tm = {}
    tic = time.time()
    sol = LSQSolver(0)
    sol.set_col_map(n_full, keep)
    tm['create_colmap'] = time.time() - tic
    tic = time.time()
    desc = describe(G_data, Gc, with_fields=True)
    tm['describe'] = time.time() - tic
    gdesc, interp, coords, stencils, npts, fields = desc
    tic = time.time()
    sol.set_matrix_stencil(int(G_data.N_eq) + int(Gc.N_eq), n_full, gdesc, interp, coords, stencils, npts,
                           fields=fields)
    tm['set_matrix_stencil'] = time.time() - tic
    from lssurf_amd.constraint_functions import node_column_blocks_affine
    tic = time.time()
    aff = node_column_blocks_affine(S['grids'], keep)
    tm['node_column_blocks_affine'] = time.time() - tic
    tic = time.time()
    sol.set_column_blocks_affine(*aff)
    tm['set_column_blocks_affine'] = time.time() - tic
    tic = time.time()
    blocks = node_column_blocks(S['grids'], keep)
    tm['node_column_blocks (explicit, for comparison)'] = time.time() - tic
    tic = time.time()
    sol.set_column_blocks_csr(*blocks)
    tm['set_column_blocks (explicit, for comparison)'] = time.time() - tic
    import numpy as np
    w = np.abs(1. / np.concatenate((S['Ed'], S['Ec'])))
    tm['formation_affine_s'] = sum(v for k, v in tm.items() if 'explicit' not in k)
    tic = time.time()
    sol.set_row_weight(w)
    tm['set_row_weight'] = time.time() - tic
    tic = time.time()
    sol.set_row_mask(np.ones(w.size, bool))
    tm['set_row_mask'] = time.time() - tic
    t2 = time.time()
    print(json.dumps({'config': cfg, 'host_assembly_s': t1 - t0, 'formation_s': t2 - t1, 'steps': tm}), flush=True)
    sol.close()


if __name__ == '__main__':
    for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 1):
        main(sys.argv[1] if len(sys.argv) > 1 else 'c4')
