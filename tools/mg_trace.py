"""Development probe: one multigrid-preconditioned CGNR solve on a BASELINE config, run twice
(the first builds the hierarchy and the iteration graph), for a rocprofv3 --kernel-trace of the
second.  `python tools/mg_trace.py analyse <kernel_trace.csv>` prints, for one CG iteration of the
last solve (between two k_cg_alpha launches), every kernel with its grid, duration and the gap
before it, and the totals per kernel name.
Usage on the GPU box: rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 tools/mg_trace.py c4"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(cfg):
    import numpy as np
    import bench
    fs, rhs, w, setup = bench.build_system(cfg, 0)
    for k in range(2):
        x, st = fs.solver.solve(rhs, precond=4, method=1)
        print(json.dumps({'config': cfg, 'pass': k, 'iters': int(st['iters']), 'time_s': st['time_s'],
                          'setup_s': st.get('setup_s', 0.0), 'xnorm': float(np.linalg.norm(x))}), flush=True)
    fs.close()


def short(name):
    for pre in ('void ', 'lsq::(anonymous namespace)::'):
        name = name.replace(pre, '')
    return name.split('(')[0]


def analyse(path, which=-3):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    al = [i for i, r in enumerate(rows) if 'k_cg_alpha' in r['Kernel_Name']]
    i0, i1 = al[which - 1], al[which]
    tot = {}
    prev_end = None
    print(f'{"kernel":40s} {"grid":>10s} {"us":>8s} {"gap":>7s}')
    for r in rows[i0:i1]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        prev_end = e
        g = int(r.get('Grid_Size_X', r.get('Grid_Size', 0)) or 0)
        nm = short(r['Kernel_Name'])
        print(f'{nm[:40]:40s} {g:10d} {(e - s) / 1e3:8.1f} {gap:7.1f}')
        t = tot.setdefault(nm, [0, 0.0])
        t[0] += 1
        t[1] += (e - s) / 1e3
    span = (int(rows[i1]['Start_Timestamp']) - int(rows[i0]['Start_Timestamp'])) / 1e3
    print(f'iteration span {span:.1f} us, kernels {i1 - i0}')
    for nm, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f'{nm[:40]:40s} {c:4d} {t:9.1f}')


def setup(path):
    """Kernels of the last solve's set-up: from the kernel after the previous solve's last CG step
    (the last k_cg_beta before the final k_cg_alpha run) to the first k_cg_alpha of the last solve."""
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    al = [i for i, r in enumerate(rows) if 'k_cg_alpha' in r['Kernel_Name']]
    # solves are separated by a gap in alpha indices larger than one iteration's kernels
    gaps = [(al[k + 1] - al[k], k) for k in range(len(al) - 1)]
    big = max(gaps)[1]
    i1 = al[big + 1]
    i0 = al[big] + 1
    while i0 < i1 and 'k_cg_beta' not in rows[i0]['Kernel_Name']:
        i0 += 1
    i0 += 1
    tot = {}
    for r in rows[i0:i1]:
        nm = short(r['Kernel_Name'])
        t = tot.setdefault(nm, [0, 0.0])
        t[0] += 1
        t[1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    span = (int(rows[i1]['Start_Timestamp']) - int(rows[i0]['Start_Timestamp'])) / 1e3
    print(f'set-up span {span:.1f} us, kernels {i1 - i0}, busy {sum(v[1] for v in tot.values()):.1f} us')
    for nm, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f'{nm[:40]:40s} {c:4d} {t:9.1f}')


if __name__ == '__main__':
    if sys.argv[1] == 'setup':
        setup(sys.argv[2])
    elif sys.argv[1] == 'analyse':
        analyse(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else -3)
    else:
        run(sys.argv[1])
