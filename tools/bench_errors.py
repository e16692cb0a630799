"""Timing of the error-propagation path (smooth_fit compute_E) on smooth_fit systems of growing
size: the banded path (lsq_cov_band: band Cholesky + rows of R⁻¹ by banded sweeps) and, up to n = 3·10⁴, the dense
device factor (lsq_sigma_x: AᵀA → Cholesky → R⁻¹ → row RSS) — development / DESIGN.md numbers.

    python tools/bench_errors.py 20 28 36 48      # nodes per side; nt = 12, 2 points per node
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import lssurf_amd as LS  # noqa: E402
from lssurf_amd import synthetic  # noqa: E402
from lssurf_amd.constraint_functions import reference_epoch_keep_cols  # noqa: E402
from lssurf_amd.smooth_fit import FitSystem  # noqa: E402


def system(S, nt=12):
    W = {'x': (S - 1) * 100., 'y': (S - 1) * 100., 't': (nt - 1) * 0.25}
    rng = np.random.default_rng(7)
    npts = 2 * S * S
    x, y = (rng.random(npts) - 0.5) * W['x'], (rng.random(npts) - 0.5) * W['y']
    t = (rng.random(npts) - 0.5) * W['t']
    z = 10 * np.sin(2 * np.pi * x / (W['x'] / 2)) + rng.normal(0, 0.1, npts)
    D = LS.containers.data().from_dict({'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(npts, 0.1)})
    return LS.smooth_fit(data=D, W=W, ctr={'x': 0., 'y': 0., 't': 0.}, spacing={'z0': 100., 'dz': 100., 'dt': 0.25},
                         E_RMS=dict(synthetic.E_RMS_NOTEBOOK), reference_epoch=nt // 2, return_fit_objects=True)


def main(sizes, dense_max=30000):
    from lssurf_amd.errors import band_order
    out = []
    for S in sizes:
        o = system(S)
        keep = reference_epoch_keep_cols(o['G_data'].col_N, o['grids']['dz'], 6)
        fs = FitSystem(o['G_data'], o['Gc'], keep, o['Gc'].col_N, device=0)
        n = keep.size
        rec = {'nodes': S, 'n': int(n)}
        try:
            w = 1. / np.concatenate([o['Ed'], o['Ec']])
            fs.solver.set_row_weight(w)
            fs.solver.set_row_mask(np.ones(fs.n_data + fs.n_con, bool))
            perm = band_order(o['grids'], keep)
            for rep in range(2):
                fs.solver.set_row_weight(w * (1 + 1e-4 * rep))      # a new factor each time
                t0 = time.time()
                Eb, _, info = fs.solver.cov_band(perm)
                rec['band_s' if rep else 'band_first_s'] = time.time() - t0
            rec.update({'band_tiles': int(info[0]), 'tile_rows': int(info[1]), 'band_bytes': int(info[2]),
                        'tile_products': int(info[3]),
                        'sweep_tflops': float(info[3]) * 2 * 64 ** 3 / rec['band_s'] / 1e12})
            if n <= dense_max:
                fs.solver.set_row_weight(w * (1 + 2e-4))
                t0 = time.time()
                Ed = fs.solver.sigma_x()
                rec['dense_s'] = time.time() - t0
                fs.solver.set_row_weight(w * (1 + 1e-4))
                Ed = fs.solver.sigma_x()
                rec['band_vs_dense_rel'] = float(np.abs(Eb - Ed).max() / np.abs(Ed).max())
        finally:
            fs.close()
        print(json.dumps(rec), flush=True)
        out.append(rec)
    return out


if __name__ == '__main__':
    main([int(a) for a in sys.argv[1:]] or [20, 28, 36])
