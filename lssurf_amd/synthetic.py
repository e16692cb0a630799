"""Synthetic point clouds for the BASELINE.json configurations.

Domain W_x = W_y = (n-1)*100 m centred on 0, spacing z0 = dz = 100 m (Z0_REFINED: z0 50 m), dt = 0.25,
W_t = (nt-1)*0.25, reference_epoch = nt//2; points uniform in (x, y, t) from
default_rng(20251121 + SEED_ID[config]); z = 10 sin(2πx/Lx) cos(2πy/Ly) + 0.5 t exp(-r²/(W/4)²)
+ N(0, 0.1), Lx = W/2, Ly = W/3, sigma = 0.1; E_RMS = notebook cell-17 set.
"""
import numpy as np

from . import containers as pc

E_RMS_NOTEBOOK = {'d2z0_dx2': 0.03, 'dz0_dx': 75., 'd3z_dx2dt': 0.006, 'd2z_dxdt': 15., 'd2z_dt2': 5000.}
E_RMS_STIFF = {'d2z0_dx2': 0.0006, 'dz0_dx': 0.9, 'd3z_dx2dt': 1e-4, 'd2z_dxdt': 0.15, 'd2z_dt2': 0.5}

# id: (nodes per side, epochs, points)   — BASELINE.json configs (C1 is the notebook-scale case)
CONFIGS = {
    'c1': (128, 9, 10_000),
    'c3': (512, 12, 1_000_000),
    'c4': (1024, 12, 2_000_000),
    'c5': (2048, 12, 8_000_000),
    # small ones for tests / smoke
    't64': (64, 12, 8_192),
    't256': (256, 12, 131_072),
    't128': (128, 12, 32_768),
    'tdense': (64, 12, 40_000),   # ~10 points per cell: strips whose point runs overflow LDS staging
    't15': (80, 15, 12_000),        # 15 epochs: the 16-long register columns; 80 nodes: two strips per row
    # one rank's window of C4 over 4 / 8 GPUs (owned node rows + 2 halo rows, 1/N of the points):
    # the per-rank compute floor of the strong-scaling runs, measurable on one GPU
    'c4y4': (1024, 12, 500_000, 258),
    'c4y8': (1024, 12, 250_000, 130),
    # one rank's window of C5 (2048²×12, 8 M points) over 8 GPUs: 256 owned rows + 2 halo rows
    'c5y8': (2048, 12, 1_000_000, 258),
    # anisotropic-constraint systems (BASELINE config C5: lssurf_amd.aniso.system3d — the z0
    # constraints are the notebook's directional operator along a circular field + magnitude)
    'c5a': (2048, 12, 8_000_000),
    'ta64': (64, 12, 8_192),
    'ta100': (100, 8, 20_000),     # two dim-1 tiles of k_cg_var2d, 13 tile rows
    # z0 on a 2× refinement of the dz lattice (spacing z0 50 m, dz 100 m: the reference notebooks'
    # setup): n dz nodes per side, 2n − 1 z0 nodes
    't64z': (64, 12, 8_192),
    'c3z': (512, 12, 1_000_000),
}
# seed offset of each config's points (default_rng(20251121 + id)): the configs' positions in
# CONFIGS when round 4 started, frozen — round 3 derived the offset from the dict position, so
# inserting 't128' moved every later config onto new points (C5a: 61 → 72 multigrid iterations
# between two builds that solve the same system alike).  New configs take new ids.
SEED_ID = {'c1': 0, 'c3': 1, 'c4': 2, 'c5': 3, 't64': 4, 't256': 5, 't128': 6, 'tdense': 7, 't15': 8,
           'c4y4': 9, 'c4y8': 10, 'c5a': 11, 'ta64': 12, 'ta100': 13, 't64z': 14, 'c3z': 15, 'c5y8': 16}
ANISO = ('c5a', 'ta64', 'ta100')
Z0_REFINED = ('t64z', 'c3z')


def config_kwargs(name, stiff=False):
    n, nt, npts = CONFIGS[name][:3]
    ny = CONFIGS[name][3] if len(CONFIGS[name]) > 3 else n   # node rows (y) when not square
    W = {'x': (n - 1) * 100., 'y': (ny - 1) * 100., 't': (nt - 1) * 0.25}
    z0s = 50. if name in Z0_REFINED else 100.
    return dict(W=W, ctr={'x': 0., 'y': 0., 't': 0.}, spacing={'z0': z0s, 'dz': 100., 'dt': 0.25},
                E_RMS=dict(E_RMS_STIFF if stiff else E_RMS_NOTEBOOK), reference_epoch=nt // 2), npts


def points(name, config_id=None):
    kw, npts = config_kwargs(name)
    cid = SEED_ID[name] if config_id is None else config_id
    rng = np.random.default_rng(20251121 + cid)
    W, ctr = kw['W'], kw['ctr']
    x = ctr['x'] + (rng.random(npts) - 0.5) * W['x']
    y = ctr['y'] + (rng.random(npts) - 0.5) * W['y']
    t = ctr['t'] + (rng.random(npts) - 0.5) * W['t']
    Lx, Ly = W['x'] / 2, W['y'] / 3
    z = 10 * np.sin(2 * np.pi * x / Lx) * np.cos(2 * np.pi * y / Ly) \
        + 0.5 * t * np.exp(-((x - ctr['x']) ** 2 + (y - ctr['y']) ** 2) / (W['x'] / 4) ** 2) \
        + rng.normal(0, 0.1, npts)
    return pc.data().from_dict({'x': x, 'y': y, 'time': t, 'z': z, 'sigma': np.full(npts, 0.1)}), kw


# 2-D z0-only configurations (BASELINE config C2: notebooks/smooth_fit_demo_aniso.ipynb style —
# interp + grad2_z0 + grad_z0 formed with lin_op and handed to the solver directly):
# id: (nodes per side, points)
CONFIGS_2D = {
    'c2': (1024, 500_000),
    't2d': (64, 4_000),
}
E_RMS_2D = {'d2z0_dx2': 0.03, 'dz0_dx': 75.}


def system2d(name):
    """(G_data, Gc, grid, row_weight, rhs) of a 2-D config: domain (n−1)·100 m square from 0,
    spacing 100 m, points uniform from default_rng(20251121 + 100 + index), z = 10 sin(2πx/L)
    cos(2πy/L') + N(0, 0.1), σ = 0.1; constraint σ = E_RMS / sqrt(cell area) as in
    constraint_functions (the structure of tests/golden sys_lin2d)."""
    from .fd_grid import fd_grid
    from .lin_op import lin_op
    n, npts = CONFIGS_2D[name]
    rng = np.random.default_rng(20251121 + 100 + list(CONFIGS_2D).index(name))
    W = (n - 1) * 100.
    g = fd_grid([[0., W], [0., W]], [100., 100.], name='z0')
    y, x = rng.uniform(0, W, npts), rng.uniform(0, W, npts)
    z = 10 * np.sin(2 * np.pi * x / (W / 2)) * np.cos(2 * np.pi * y / (W / 3)) + rng.normal(0, 0.1, npts)
    sigma = np.full(npts, 0.1)
    G = lin_op(g, name='interp_z').interp_mtx([y, x])
    root = np.sqrt(np.prod(g.delta))
    g2 = lin_op(g, name='grad2_z0').grad2(DOF='z0')
    g2.expected = E_RMS_2D['d2z0_dx2'] / root * np.ones(g2.N_eq)
    g1 = lin_op(g, name='grad_z0').grad(DOF='z0')
    g1.expected = E_RMS_2D['dz0_dx'] / root * np.ones(g1.N_eq)
    Gc = lin_op(None, name='constraints').vstack([g2, g1])
    E_all = np.concatenate([sigma, g2.expected, g1.expected])
    rhs = np.concatenate([z, np.zeros(Gc.N_eq)])
    return G, Gc, g, 1. / E_all, rhs


def aniso_system(name, stiff=False, config_id=None):
    """lssurf_amd.aniso.system3d on the synthetic points of an anisotropic config (ANISO)."""
    from . import aniso
    D, kw = points(name, config_id)
    if stiff:
        kw['E_RMS'] = dict(E_RMS_STIFF)
    return aniso.system3d(D, **kw), kw
