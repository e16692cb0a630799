"""Host (scipy) multigrid hierarchy for the GPU tests of precond 4 (lssurf_amd/csrc/mg.inc): the
same prolongation (bilinear in (y, x), coarse node a on fine node 2a, identity in t), Galerkin
stencil operators PᵀN_sP and (y, x)-lumped data operators, built from the formed A the device
returns.  Test infrastructure only."""
import numpy as np
import scipy.sparse as sp


def prolong1(nf):
    """1-D prolongation fine (nf) <- coarse (nf // 2 + 1)."""
    nc = nf // 2 + 1
    r, c, v = [], [], []
    for i in range(nf):
        if i % 2 == 0:
            r.append(i)
            c.append(i // 2)
            v.append(1.0)
        else:
            r += [i, i]
            c += [(i - 1) // 2, (i + 1) // 2]
            v += [0.5, 0.5]
    return sp.csr_matrix((v, (r, c)), shape=(nf, nc))


def prolong_full(ny, nx, nt):
    """Full-space prolongation of the [z0 (ny·nx); dz (ny·nx·nt)] column layout."""
    Py, Px = prolong1(ny), prolong1(nx)
    P2 = sp.kron(Py, Px).tocsr()
    P3 = sp.kron(P2, sp.identity(nt)).tocsr()
    return sp.block_diag([P2, P3]).tocsr(), Py.shape[1], Px.shape[1]


def node_of(ny, nx, nt):
    nodes = np.arange(ny * nx)
    return np.concatenate([nodes, np.repeat(nodes, nt)])


def slot_of(ny, nx, nt):
    return np.concatenate([np.zeros(ny * nx, int), 1 + np.tile(np.arange(nt), ny * nx)])


def lump_by_node(D, node, slot):
    """Move entry (i, j) to (i, j') with j' = the column of node(i) holding slot(j)."""
    Dc = D.tocoo()
    n = D.shape[0]
    table = np.full((node.max() + 1, slot.max() + 1), -1)
    table[node, slot] = np.arange(n)
    jn = table[node[Dc.row], slot[Dc.col]]
    ok = jn >= 0
    return sp.csr_matrix((Dc.data[ok], (Dc.row[ok], jn[ok])), shape=D.shape)


def hierarchy(A, n_data_rows, keep_cols, ny, nx, nt, coarse=5, coarse_cols=1024):   # mg.inc MG_COARSE, MG_COARSE_COLS
    """Levels [(shape, keep_mask_full, N_operator_full)] with N over each level's FULL column
    space (rows / columns of removed epochs zero).  Level 0: AᵀA; coarse: Galerkin stencil part +
    lumped data part."""
    n_full = ny * nx * (1 + nt)
    keep = np.zeros(n_full, bool)
    keep[keep_cols] = True
    E = sp.csr_matrix((np.ones(keep_cols.size), (keep_cols, np.arange(keep_cols.size))),
                      shape=(n_full, keep_cols.size))       # compact -> full
    Ad, As = A[:n_data_rows], A[n_data_rows:]
    Ns = (E @ (As.T @ As) @ E.T).tocsr()
    Nd = (E @ (Ad.T @ Ad) @ E.T).tocsr()
    levels = [((ny, nx), keep, (Ns + Nd).tocsr())]
    while max(ny, nx) > coarse and not (len(levels) > 1 and ny * nx * (1 + nt) <= coarse_cols):
        P, nyc, nxc = prolong_full(ny, nx, nt)
        Ns = (P.T @ Ns @ P).tocsr()
        Nd = lump_by_node((P.T @ Nd @ P).tocsr(), node_of(nyc, nxc, nt), slot_of(nyc, nxc, nt))
        kc = np.concatenate([np.ones(nyc * nxc, bool), np.tile(keep[ny * nx:ny * nx + nt], nyc * nxc)])
        Dk = sp.diags(kc.astype(float))
        ny, nx, keep = nyc, nxc, kc
        levels.append(((ny, nx), keep, (Dk @ (Ns + Nd) @ Dk).tocsr()))
    return levels
