"""Development probe: is lsq_cov_band deterministic and equal to the dense path at t64?"""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ewin_probe import system  # noqa: E402
from lssurf_amd.errors import band_order  # noqa: E402
name = sys.argv[1] if len(sys.argv) > 1 else 't64'
S, fs, keep = system(name)
o = band_order(S['grids'], keep)
E1, _, i1 = fs.solver.cov_band(o)
E2, _, i2 = fs.solver.cov_band(o)
E3, _, i3 = fs.solver.cov_band_window(o)
Ed = fs.solver.sigma_x()
r = lambda a, b: float(np.max(np.abs(a - b) / b))
print(json.dumps({'E1-E2': r(E1, E2), 'E1-dense': r(E1, Ed), 'E2-dense': r(E2, Ed), 'E3-dense': r(E3, Ed),
                  'info': i1.tolist()}))
fs.close()
# the factor itself, twice
S, fs, keep = system(name)
R1, p1 = fs.solver.band_factor(o)
R2, p2 = fs.solver.band_factor(o)
d = abs(R1 - R2)
print(json.dumps({'factor max diff': float(d.max()) if d.nnz else 0.0, 'factor max': float(abs(R1).max())}))
fs.close()
