"""cProfile of smooth_fit end to end (development): python tools/profile_e2e.py c4 3"""
import cProfile
import pstats
import sys
import time

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import lssurf_amd as LS  # noqa: E402
from lssurf_amd import synthetic  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'c4'
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
D, kw = synthetic.points(cfg)
LS.smooth_fit(data=synthetic.points('t64')[0], VERBOSE=False, max_iterations=1, **synthetic.config_kwargs('t64')[0])
pr = cProfile.Profile()
t0 = time.time()
pr.enable()
S = LS.smooth_fit(data=D, VERBOSE=False, max_iterations=iters, **kw)
pr.disable()
print('wall', time.time() - t0, {k: v for k, v in S['timing'].items() if not isinstance(v, dict)})
pstats.Stats(pr).sort_stats('cumulative').print_stats(45)
pstats.Stats(pr).sort_stats('tottime').print_stats(25)
