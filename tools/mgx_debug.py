"""Development probe: the z0-refined multigrid on a golden system (operator, V-cycle symmetry, λ,
PCG iterations and error against the golden x)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from test_gpu_cgnr import _golden_system, TOL
name = sys.argv[1]
g, fs, w, rhs = _golden_system(name)
fs.solver.set_row_weight(w)
fs.solver.set_row_mask(np.ones(fs.n_data + fs.n_con, bool))
print('cg4', fs.solver.cg_available(4))
levels, tref = fs.solver.mg_info()
print('levels', levels, 'tref', tref, 'n_full', fs.n_full, 'keep', fs.keep_cols.size)
lam = fs.solver.mg_apply(0, 2)
print('lam0', lam)
rng = np.random.default_rng(1)
nf = fs.n_full
km = np.zeros(nf, bool); km[fs.keep_cols] = True
A = fs.solver.get_csr()
x = np.where(km, rng.standard_normal(nf), 0.0)
y = fs.solver.mg_apply(0, 0, x)
yr = np.zeros(nf); yr[fs.keep_cols] = A.T @ (A @ x[fs.keep_cols])
print('op err', np.abs(y - yr).max() / np.abs(yr).max())
u = np.where(km, rng.standard_normal(nf), 0.0); v = np.where(km, rng.standard_normal(nf), 0.0)
Vu, Vv = fs.solver.mg_apply(0, 1, u), fs.solver.mg_apply(0, 1, v)
print('sym', v @ Vu, u @ Vv, 'pd', u @ Vu, v @ Vv, 'nonkept', np.abs(Vu[~km]).max())
N = (A.T @ A).toarray()
# preconditioned operator spectrum: V ≈ N^-1 ?
idx = fs.keep_cols
M = np.zeros((idx.size, idx.size))
for j in range(min(idx.size, 4000)):
    e = np.zeros(nf); e[idx[j]] = 1.0
    M[:, j] = fs.solver.mg_apply(0, 1, e)[idx]
if idx.size <= 4000:
    ev = np.linalg.eigvals(M @ N)
    print('eig(VN) min/max real', ev.real.min(), ev.real.max(), 'max imag', np.abs(ev.imag).max())
    print('V symmetric err', np.abs(M - M.T).max() / np.abs(M).max())
xm = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=4, method=1, maxit=5000, **TOL)
print('mg stats', fs.stats)
print('rel err', np.linalg.norm(xm - g['x']) / np.linalg.norm(g['x']))
xb = fs.solve(w, np.ones(fs.n_data, bool), rhs, precond=3, method=1, maxit=50000, **TOL)
print('bj stats', fs.stats['iters'], 'rel err', np.linalg.norm(xb - g['x']) / np.linalg.norm(g['x']))
fs.close()
