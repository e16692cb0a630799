"""cProfile of smooth_fit end to end at a bench config (host-side hot spots): prints the top
functions by cumulative and by own time.  python tools/profile_e2e.py c4 3"""
import cProfile
import pstats
import sys
import time

sys.path.insert(0, '.')
import lssurf_amd as LS                 # noqa: E402
from lssurf_amd import synthetic        # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else 'c4'
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
D, kw = synthetic.points(config)
LS.smooth_fit(data=D, VERBOSE=False, max_iterations=1, **kw)   # warm: library load, first-touch
pr = cProfile.Profile()
t0 = time.time()
pr.enable()
S = LS.smooth_fit(data=D, VERBOSE=False, max_iterations=iters, **kw)
pr.disable()
print(f'wall {time.time() - t0:.3f} s', flush=True)
st = pstats.Stats(pr)
st.sort_stats('cumulative').print_stats(45)
st.sort_stats('tottime').print_stats(30)
