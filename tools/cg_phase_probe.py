"""Development probe: per-kernel times of one CGNR iteration (block-Jacobi) on a BASELINE config.
Tuning variables the library reads when it builds the normal-stencil description (e.g.
LSQ_CG_RPW) are taken from the environment, so run one process per setting.
Usage: python tools/cg_phase_probe.py [config]  — prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'c4'
fs, rhs, w, setup = bench.build_system(cfg, 0)
p = fs.solver.profile_cg(reps=10, precond=3)
env = {k: v for k, v in os.environ.items() if k.startswith('LSQ_CG')}
print(json.dumps({'config': cfg, 'env': env, **{k: v for k, v in p.items() if k != 'bytes'}}), flush=True)
fs.close()
