"""Development prototype (SURVEY §8(f) row 2 option iii): a probing estimator of
diag((AᵀA)⁻¹) on multigrid PCG, measured against the exact band covariance (`lsq_cov_band`).

Colouring by node distance: the columns of one slot (z0, or dz at one epoch) on the nodes
(iy, ix) with iy ≡ a, ix ≡ b (mod D) form one colour; the probe v = Σ_{j ∈ colour} e_j, and
x = N⁻¹v read at the colour's columns estimates (N⁻¹)_jj up to the correlations between columns D
or more nodes apart.  D² × (slots) probes, each one PCG solve of N x = v with the V-cycle
(N through `lsq_normal_apply`, the V-cycle through `lsq_mg_apply`: host round trips, fine at the
validation sizes).  Prints per spacing D: probes, PCG iterations, the relative error of
sqrt(diag) against the band (max / 99th percentile / median) and the C4 cost the probe count
implies at one multigrid solve per probe (C4 solve time given on the command line).

    python tools/probe_diag.py t64 4,8,16 0.14"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])


def pcg(fs, kmask, v, tol=1e-10, maxit=500):
    """N x = v on the kept columns, preconditioned by one V-cycle."""
    x = np.zeros_like(v)
    r = v.copy()
    z = fs.solver.mg_apply(0, 1, r) * kmask
    p = z.copy()
    rz = r @ z
    r0 = np.sqrt(r @ r)
    for it in range(1, maxit + 1):
        q = fs.solver.normal_apply(p) * kmask
        a = rz / (p @ q)
        x += a * p
        r -= a * q
        if np.sqrt(r @ r) <= tol * r0:
            return x, it
        z = fs.solver.mg_apply(0, 1, r) * kmask
        rz_new = r @ z
        p = z + (rz_new / rz) * p
        rz = rz_new
    return x, maxit


def main(cfg, spacings, c4_solve_s):
    import lssurf_amd as LS
    from lssurf_amd import synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    from lssurf_amd.errors import band_order
    from lssurf_amd.smooth_fit import FitSystem
    D_, kw = synthetic.points(cfg)
    S = LS.smooth_fit(data=D_, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, grids=S['grids'])
    try:
        w = np.abs(1. / np.concatenate((S['Ed'], S['Ec'])))
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.ones(w.size, bool))
        ok, why = fs.solver.cg_available(4)
        assert ok, why
        t0 = time.time()
        E_band, _, _ = fs.solver.cov_band(band_order(S['grids'], fs.keep_cols))
        t_band = time.time() - t0
        nf = fs.n_full
        kmask = np.zeros(nf)
        kmask[fs.keep_cols] = 1.0
        z0, dz = S['grids']['z0'], S['grids']['dz']
        ny, nx, nt = (int(s) for s in dz.shape)
        iy, ix = np.divmod(np.arange(ny * nx), nx)
        slots = [z0.col_0 + np.arange(ny * nx)] + [dz.col_0 + np.arange(ny * nx) * nt + t for t in range(nt)]
        pos = np.full(nf, -1)
        pos[fs.keep_cols] = np.arange(fs.keep_cols.size)
        for D in spacings:
            est = np.zeros(fs.keep_cols.size)
            iters, probes = [], 0
            t0 = time.time()
            for cols in slots:
                if pos[cols[0]] < 0:
                    continue   # removed epoch
                for a in range(D):
                    for b in range(D):
                        sel = cols[(iy % D == a) & (ix % D == b)]
                        v = np.zeros(nf)
                        v[sel] = 1.0
                        x, it = pcg(fs, kmask, v)
                        est[pos[sel]] = x[sel]
                        iters.append(it)
                        probes += 1
                        if probes % 256 == 0:
                            print(f'... D={D} {probes} probes {time.time() - t0:.0f} s', flush=True)
            rel = np.abs(np.sqrt(np.maximum(est, 0)) - E_band) / E_band
            print(json.dumps({'config': cfg, 'D': D, 'probes': probes, 'pcg_iters_mean': float(np.mean(iters)),
                              'rel_err_max': float(rel.max()), 'rel_err_p99': float(np.quantile(rel, 0.99)),
                              'rel_err_median': float(np.median(rel)), 'wall_s': time.time() - t0,
                              'band_s': t_band, 'c4_cost_s_at_one_solve_per_probe': probes * c4_solve_s}),
                  flush=True)
    finally:
        fs.close()


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 't64',
         [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else '4,8').split(',')],
         float(sys.argv[3]) if len(sys.argv) > 3 else 0.14)
