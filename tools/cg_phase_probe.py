"""Development probe: per-phase cost of the CGNR normal-stencil kernel on a BASELINE config.
LSQ_CG_DBG bits: 1 skip the stencil compute, 4 skip the staging loads, 8 skip the q stores,
16 replace the stencil sum by the centre value.  Prints one JSON line per mode."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'c4'
fs, rhs, w, setup = bench.build_system(cfg, 0)
for mode in [int(a) for a in sys.argv[2:]] or (0, 1, 4, 5):
    os.environ['LSQ_CG_DBG'] = str(mode)
    p = fs.solver.profile_cg(reps=10, precond=3)
    print(json.dumps({'mode': mode, **{k: v for k, v in p.items() if k != 'bytes'}}), flush=True)
fs.close()
