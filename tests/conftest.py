import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) and liblsqsurf.so')


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def golden_csr(g, prefix='A'):
    return sp.csr_matrix((g[prefix + '_data'], g[prefix + '_indices'], g[prefix + '_indptr']),
                         shape=tuple(g[prefix + '_shape']))


def golden_points(g):
    from lssurf_amd import containers as pc
    return pc.data().from_dict({k[3:]: g[k] for k in g.files if k.startswith('in_') and not k.startswith('in_mask_')})


def golden_avg_masks(g):
    """the named avg_masks region of sys_avg.npz as a grid container"""
    from lssurf_amd import containers as pc
    return {'basin': pc.grid.data().from_dict({'x': g['in_mask_x'], 'y': g['in_mask_y'], 'z': g['in_mask_z']})}


def golden_kwargs(g):
    import ast
    return ast.literal_eval(str(g['kwargs']))


SYSTEMS = ['sf3d', 'sf3d_edit', 'nb_xt', 'nb_err', 'sf3d_eq_edit']


@pytest.fixture(scope='session')
def gpu_available():
    try:
        from lssurf_amd.solver import LSQSolver
        LSQSolver(0).close()
        return True
    except Exception as e:   # noqa: BLE001
        pytest.fail(f'GPU test requested but the device path is unavailable: {e}')
