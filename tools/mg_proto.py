"""Design experiment (CPU, scipy): PCG iteration counts on the smooth_fit normal equations with
block-Jacobi vs a geometric multigrid V-cycle (Galerkin coarse operators PᵀNP, bilinear (y, x)
prolongation, identity in t, Chebyshev/block-Jacobi smoothing).  Not product code.

usage: python tools/mg_proto.py t64|t256|c1 [tol]
"""
import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.linalg as sla

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import lssurf_amd as LS  # noqa: E402
from lssurf_amd import synthetic  # noqa: E402
from lssurf_amd.constraint_functions import reference_epoch_keep_cols, node_column_blocks  # noqa: E402


def system(cfg):
    D, kw = synthetic.points(cfg)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    G = sp.vstack([S['G_data'].toCSR(), S['Gc'].toCSR()]).tocsr()
    G = sp.csr_matrix(G, shape=(G.shape[0], S['Gc'].col_N))
    w = 1. / np.concatenate((S['Ed'], S['Ec']))
    A = (sp.diags(w) @ G)[:, keep].tocsr()
    b = w * np.concatenate([S['data'].z, np.zeros(S['Gc'].N_eq)])
    return A, b, keep, S['grids'], S['G_data'].N_eq


def prolong1(nf):
    nc = nf // 2 + 1
    r, c, v = [], [], []
    for i in range(nf):
        if i % 2 == 0:
            r.append(i); c.append(i // 2); v.append(1.0)
        else:
            r += [i, i]; c += [(i - 1) // 2, (i + 1) // 2]; v += [0.5, 0.5]
    return sp.csr_matrix((v, (r, c)), shape=(nf, nc))


def blocks_of(ny, nx, nt, keep_local):
    """node blocks in a [z0 (ny nx); dz (ny nx nt)] space restricted to keep_local (ascending)."""
    class G:
        pass
    z0 = G(); z0.shape = (ny, nx); z0.col_0 = 0; z0.ctrs = [np.arange(ny), np.arange(nx)]; z0.N_dims = 2
    dz = G(); dz.shape = (ny, nx, nt); dz.col_0 = ny * nx; dz.ctrs = [np.arange(ny), np.arange(nx), np.arange(nt)]
    dz.N_dims = 3
    return node_column_blocks({'z0': z0, 'dz': dz}, keep_local)


class BJ:
    def __init__(self, N, ptr, cols):
        self.ptr, self.cols = ptr, cols
        Nc = N.tocsr()
        k = ptr[1] - ptr[0]
        assert np.all(np.diff(ptr) == k)
        nb = ptr.size - 1
        C = cols.reshape(nb, k)
        self.C = C
        blk = np.empty((nb, k, k))
        for i in range(k):
            for j in range(k):
                blk[:, i, j] = np.asarray(Nc[C[:, i], C[:, j]]).ravel()
        self.inv = np.linalg.inv(blk)

    def __call__(self, r):
        z = np.empty_like(r)
        z[self.C] = np.einsum('bij,bj->bi', self.inv, r[self.C])
        return z


POWER_ITS = 10


def power_max(N, M, n, its=None, rng=np.random.default_rng(0)):
    """Rayleigh quotient of M⁻¹N in the M inner product (the device recipe): v M-normalised,
    q = N v, λ = v·q, w = M⁻¹q, v ← w / sqrt(w·q)."""
    its = its or POWER_ITS
    v = rng.standard_normal(n)
    lam = 0
    for k in range(its):
        q = N @ v
        if k:
            lam = max(lam, v @ q)
        w = M(q)
        v = w / np.sqrt(w @ q)
    return lam


class Level:
    pass


def node_of_cols(ny, nx, nt, keep_mask):
    """node id of every kept column of a [z0; dz] space"""
    nodes = np.concatenate([np.arange(ny * nx), np.repeat(np.arange(ny * nx), nt)])
    return nodes[keep_mask]


def lump_by_node(D, node):
    """block-lump a column-space operator over (y, x) neighbours: entry (i, j) moves to
    (i, j') where j' is the column of node(i) with j's slot; returns the lumped operator."""
    # slot of a column within its node: position among the node's columns
    Dc = D.tocoo()
    n = D.shape[0]
    order = np.lexsort((np.arange(n), node))
    slot = np.empty(n, int)
    # columns of a node are contiguous in order; slot = rank within node
    nd_sorted = node[order]
    starts = np.r_[0, np.flatnonzero(np.diff(nd_sorted)) + 1]
    rank = np.arange(n) - np.repeat(starts, np.diff(np.r_[starts, n]))
    slot[order] = rank
    nslots = rank.max() + 1
    table = np.full((node.max() + 1, nslots), -1)
    table[node, slot] = np.arange(n)
    jn = table[node[Dc.row], slot[Dc.col]]
    ok = jn >= 0
    return sp.csr_matrix((Dc.data[ok], (Dc.row[ok], jn[ok])), shape=D.shape)


def build_levels(A, keep, grids, coarse_max=2500, lo_frac=0.1, deg=2, lump=False, n_data=None):
    ny, nx, nt = grids['dz'].shape
    nf_full = ny * nx * (1 + nt)
    keep_mask = np.zeros(nf_full, bool)
    keep_mask[keep] = True
    N = (A.T @ A).tocsr()
    if lump:
        Ad, As = A[:n_data], A[n_data:]
        Ns = (As.T @ As).tocsr()
        Nd = (Ad.T @ Ad).tocsr()
    levels = []
    while True:
        L = Level()
        L.N = N
        L.n = N.shape[0]
        L.shape = (ny, nx, nt)
        keep_idx = np.flatnonzero(keep_mask)
        if L.n <= coarse_max:
            L.chol = sla.cho_factor(N.toarray())
            levels.append(L)
            break
        ptr, cols = blocks_of(ny, nx, nt, keep_idx)
        L.M = BJ(N, ptr, cols)
        lmax = power_max(N, L.M, L.n)
        L.lmax = 1.1 * lmax
        L.lmin = lo_frac * lmax
        L.deg = deg
        # prolongation (full coarse -> full fine), then restricted to kept
        Py, Px = prolong1(ny), prolong1(nx)
        nyc, nxc = Py.shape[1], Px.shape[1]
        P2 = sp.kron(Py, Px).tocsr()
        P3 = sp.kron(P2, sp.identity(nt)).tocsr()
        P = sp.block_diag([P2, P3]).tocsr()
        keep_c = np.zeros(nyc * nxc * (1 + nt), bool)
        keep_c[:nyc * nxc] = True
        kc3 = keep_mask[ny * nx:].reshape(ny * nx, nt)[0]
        keep_c[nyc * nxc:] = np.tile(kc3, nyc * nxc)
        L.P = P[keep_mask][:, keep_c].tocsr()
        levels.append(L)
        if lump:
            Ns = (L.P.T @ Ns @ L.P).tocsr()
            Nd = lump_by_node((L.P.T @ Nd @ L.P).tocsr(), node_of_cols(nyc, nxc, nt, keep_c))
            N = (Ns + Nd).tocsr()
        else:
            N = (L.P.T @ N @ L.P).tocsr()
        ny, nx = nyc, nxc
        keep_mask = keep_c
    return levels


def cheb(L, r, x=None):
    """Chebyshev smoothing of N x = r with block-Jacobi, deg steps, from x (or 0)."""
    N, M = L.N, L.M
    theta = 0.5 * (L.lmax + L.lmin)
    delta = 0.5 * (L.lmax - L.lmin)
    sigma = theta / delta
    x = np.zeros_like(r) if x is None else x.copy()
    res = r - N @ x if x.any() else r.copy()
    rho = 1.0 / sigma
    d = M(res) / theta
    for k in range(L.deg):
        x += d
        if k == L.deg - 1:
            break
        res -= N @ d
        rho_new = 1.0 / (2 * sigma - rho)
        d = rho_new * rho * d + (2 * rho_new / delta) * M(res)
        rho = rho_new
    return x


def vcycle(levels, l, r):
    L = levels[l]
    if hasattr(L, 'chol'):
        return sla.cho_solve(L.chol, r)
    x = cheb(L, r)
    rr = r - L.N @ x
    x += L.P @ vcycle(levels, l + 1, L.P.T @ rr)
    x = cheb(L, r, x)
    return x


def pcg(N, b, M, tol, maxit=5000):
    x = np.zeros_like(b)
    s = b.copy()
    z = M(s)
    p = z.copy()
    rho = s @ z
    s0 = np.linalg.norm(s)
    for it in range(1, maxit + 1):
        q = N @ p
        a = rho / (p @ q)
        x += a * p
        s -= a * q
        if np.linalg.norm(s) <= tol * s0:
            return x, it
        z = M(s)
        rn = s @ z
        p = z + (rn / rho) * p
        rho = rn
    return x, maxit


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else 't64'
    tol = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-10
    t0 = time.time()
    A, b, keep, grids, n_data = system(cfg)
    N = (A.T @ A).tocsr()
    rhs = A.T @ b
    print(f'{cfg}: m={A.shape[0]} n={A.shape[1]} setup {time.time() - t0:.1f}s', flush=True)
    ny, nx, nt = grids['dz'].shape
    ptr, cols = blocks_of(ny, nx, nt, keep)
    t0 = time.time()
    x_bj, it_bj = pcg(N, rhs, BJ(N, ptr, cols), tol)
    print(f'block-Jacobi PCG: {it_bj} iterations ({time.time() - t0:.1f}s)', flush=True)
    for lump in (False, True):
        for deg in (1, 2):
            lo = 0.1
            t0 = time.time()
            levels = build_levels(A, keep, grids, lo_frac=lo, deg=deg, lump=lump, n_data=n_data)
            x_mg, it_mg = pcg(N, rhs, lambda r: vcycle(levels, 0, r), tol)
            rel = np.linalg.norm(x_mg - x_bj) / np.linalg.norm(x_bj)
            print(f'MG lump={lump} deg={deg} lo={lo}: {len(levels)} levels, {it_mg} iterations, rel diff {rel:.1e} '
                  f'({time.time() - t0:.1f}s)', flush=True)


if __name__ == '__main__':
    main()
