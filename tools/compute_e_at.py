"""compute_E at a BASELINE size (development): smooth_fit(compute_E=True, max_iterations=1) on the
synthetic point cloud of `config`; prints the timing breakdown (solve, E windows, the window
self-check) as one JSON line.  A heartbeat line every 60 s keeps the GPU runner's watchdog fed.

    python tools/compute_e_at.py c4"""
import json
import sys
import threading
import time

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])


def beat(stop):
    t0 = time.time()
    while not stop.wait(60):
        print(f'... {time.time() - t0:.0f} s', flush=True)


def main(cfg):
    import lssurf_amd as LS
    from lssurf_amd import synthetic
    D, kw = synthetic.points(cfg)
    stop = threading.Event()
    threading.Thread(target=beat, args=(stop,), daemon=True).start()
    t0 = time.time()
    S = LS.smooth_fit(data=D, VERBOSE=False, max_iterations=1, compute_E=True, **kw)
    wall = time.time() - t0
    stop.set()
    tim = {k: v for k, v in S['timing'].items() if not isinstance(v, dict) or k.startswith('E_')}
    sz = S['E']['sigma_z0'].sigma_z0
    import hashlib
    import numpy as np
    digest = hashlib.sha256(np.ascontiguousarray(np.asarray(sz, dtype=np.float64)).tobytes()).hexdigest()[:16]
    import os
    if os.environ.get('LSQ_E_SAVE'):   # σ grids for a comparison between switches (npz)
        np.savez(os.environ['LSQ_E_SAVE'], sigma_z0=np.asarray(sz), sigma_dz=np.asarray(S['E']['sigma_dz'].sigma_dz))
    print(json.dumps({'config': cfg, 'wall_s': wall, 'timing': tim,
                      'sigma_z0_median': float(sorted(sz.ravel())[sz.size // 2]),
                      'sigma_z0_sha16': digest,   # bit-level identity of σ_z0 between builds / switches
                      'approximate': getattr(S['E']['sigma_z0'], 'approximate', None)}, default=float), flush=True)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'c4')
