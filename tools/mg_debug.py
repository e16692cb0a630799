"""GPU diagnostic (development): where a multigrid level operator differs from the host
hierarchy — by column kind (z0 / dz epoch), by node position, stencil vs data part."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0] + '/tests')
from mg_host import prolong_full, lump_by_node, node_of, slot_of  # noqa: E402
from test_gpu_cgnr import _synthetic_system  # noqa: E402
import scipy.sparse as sp  # noqa: E402


def main(which='t64', level=1):
    S, fs, w, rhs = _synthetic_system(which)
    keep = np.ones(fs.n_data, bool)
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.concatenate([keep, np.ones(fs.n_con, bool)]))
    print(fs.solver.cg_available(4))
    levels, tref = fs.solver.mg_info()
    print('levels', levels, 'tref', tref)
    A = fs.solver.get_csr()
    ny, nx, nt = S['grids']['dz'].shape
    n_full = ny * nx * (1 + nt)
    E = sp.csr_matrix((np.ones(fs.keep_cols.size), (fs.keep_cols, np.arange(fs.keep_cols.size))),
                      shape=(n_full, fs.keep_cols.size))
    nd = int(keep.sum())
    Ns = (E @ (A[nd:].T @ A[nd:]) @ E.T).tocsr()
    Nd = (E @ (A[:nd].T @ A[:nd]) @ E.T).tocsr()
    kmask = np.zeros(n_full, bool)
    kmask[fs.keep_cols] = True
    for l in range(level):
        P, nyc, nxc = prolong_full(ny, nx, nt)
        Ns = (P.T @ Ns @ P).tocsr()
        Nd = lump_by_node((P.T @ Nd @ P).tocsr(), node_of(nyc, nxc, nt), slot_of(nyc, nxc, nt))
        kmask = np.concatenate([np.ones(nyc * nxc, bool), np.tile(kmask[ny * nx:ny * nx + nt], nyc * nxc)])
        ny, nx = nyc, nxc
    Dk = sp.diags(kmask.astype(float))
    Ns, Nd = Dk @ Ns @ Dk, Dk @ Nd @ Dk
    rng = np.random.default_rng(1)
    nf = kmask.size
    nodes = ny * nx
    for kind in ('z0', 'dz', 'all'):
        x = np.where(kmask, rng.standard_normal(nf), 0.0)
        if kind == 'z0':
            x[nodes:] = 0
        elif kind == 'dz':
            x[:nodes] = 0
        y = fs.solver.mg_apply(level, 0, x)
        ys, yd = Ns @ x, Nd @ x
        e = y - ys - yd
        print(kind, 'rel err', np.abs(e).max() / np.abs(ys + yd).max(),
              '| err vs data-only', np.abs(y - ys).max() / np.abs(yd).max(),
              '| err vs stencil-only', np.abs(y - yd).max() / np.abs(ys).max())
        ez, ed = e[:nodes].reshape(ny, nx), e[nodes:].reshape(ny, nx, nt)
        print('  z0 err max', np.abs(ez).max(), 'dz err max by t', np.abs(ed).max(axis=(0, 1)).round(6))
        print('  z0 err rows', np.abs(ez).max(axis=1).round(4)[:12], '...')
        print('  z0 err cols', np.abs(ez).max(axis=0).round(4)[:12], '...')
        print('  dz err rows', np.abs(ed).max(axis=(1, 2)).round(4)[:12], '...')
        print('  dz err cols', np.abs(ed).max(axis=(0, 2)).round(4)[:12], '...')
    fs.close()




def unit(which='t64', level=1, node=None):
    S, fs, w, rhs = _synthetic_system(which)
    keep = np.ones(fs.n_data, bool)
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.concatenate([keep, np.ones(fs.n_con, bool)]))
    levels, tref = fs.solver.mg_info()
    A = fs.solver.get_csr()
    ny, nx, nt = S['grids']['dz'].shape
    n_full = ny * nx * (1 + nt)
    E = sp.csr_matrix((np.ones(fs.keep_cols.size), (fs.keep_cols, np.arange(fs.keep_cols.size))),
                      shape=(n_full, fs.keep_cols.size))
    nd = int(keep.sum())
    Nd = (E @ (A[:nd].T @ A[:nd]) @ E.T).tocsr()
    Ns = (E @ (A[nd:].T @ A[nd:]) @ E.T).tocsr()
    for l in range(level):
        P, nyc, nxc = prolong_full(ny, nx, nt)
        Ns = (P.T @ Ns @ P).tocsr()
        Nd = lump_by_node((P.T @ Nd @ P).tocsr(), node_of(nyc, nxc, nt), slot_of(nyc, nxc, nt))
        ny, nx = nyc, nxc
    nodes = ny * nx
    m = node if node is not None else (ny // 2) * nx + nx // 2
    x = np.zeros(nodes * (1 + nt))
    x[m] = 1.0
    y = fs.solver.mg_apply(level, 0, x)
    yd, ys = Nd @ x, Ns @ x
    cols = nodes + m * nt + np.arange(nt)
    print('node', m, 'z0 row: dev', y[m], 'host', yd[m] + ys[m])
    print('dz rows dev :', y[cols].round(4))
    print('dz rows host:', (yd + ys)[cols].round(4))
    nz = np.flatnonzero(np.abs(y - yd - ys) > 1e-9 * np.abs(yd + ys).max())
    print('mismatch columns', nz[:20], 'of', nz.size)
    fs.close()


if __name__ == "__main__" and len(sys.argv) > 3:
    unit(sys.argv[1], int(sys.argv[2]))
elif __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else 't64', int(sys.argv[2]) if len(sys.argv) > 2 else 1)
