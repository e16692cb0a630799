"""Development: one multigrid-PCG iteration's kernels (name, grid, µs, gap before) from a
rocprofv3 --kernel-trace CSV of `bench.py` (the bench's multigrid solve), plus the per-kernel sums
over that iteration.  Usage: python tools/mg_iter_trace.py run_kernel_trace.csv [which]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r'lsq::\(anonymous namespace\)::', '', name)
    name = re.sub(r'^void ', '', name)
    m = re.match(r'([^(]+)', name)
    return m.group(1).strip()


def main(path, which=-1):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    k = [(short(r['Kernel_Name']), int(r['Grid_Size_X']), int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows]
    # iterations of the multigrid solves: from one k_cg_beta (the end of a CG step) to the next,
    # with k_mg_ kernels between (α has no launch of its own since round 4's closing commit)
    starts = [i + 1 for i, e in enumerate(k) if e[0] == 'k_cg_beta']
    its = [(a, b) for a, b in zip(starts, starts[1:]) if any(e[0].startswith('k_mg_') for e in k[a:b])
           and max(e[3] - e[2] for e in k[a:b] if e[0].startswith('k_cg_normal')) > 30_000   # live (not stopped)
           and not any(e[0] in ('k_block_factor', 'k_mg_power_scalar') for e in k[a:b])]     # no per-solve set-up
    print(f'{len(its)} multigrid iterations in the trace')
    a, b = its[which if which >= 0 else len(its) // 2]
    tot = defaultdict(lambda: [0, 0.0])
    print(f"{'kernel':44s} {'grid':>9s} {'us':>8s} {'gap':>7s}")
    prev = None
    for name, g, s, e in k[a:b]:
        gap = (s - prev) / 1e3 if prev else 0.0
        print(f'{name[:44]:44s} {g:9d} {(e - s) / 1e3:8.1f} {gap:7.1f}')
        tot[name][0] += 1
        tot[name][1] += (e - s) / 1e3
        prev = e
    span = (k[b][2] - k[a][2]) / 1e3
    print(f'iteration span {span:.1f} us, kernels {b - a}, kernel sum {sum(v[1] for v in tot.values()):.1f} us')
    for name, (n, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f'{name[:44]:44s} {n:3d} {us:9.1f}')


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else -1)
