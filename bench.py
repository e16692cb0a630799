#!/usr/bin/env python3
"""bench.py — LSQR iterations/s (+ solve wall time) of the smooth_fit least-squares system on
MI355X, BASELINE.json metric.  Default workload: configs[3] = 1024x1024x12 fd_grid, 2 M points.

A "step" = one LSQR iteration on the device-resident system (SpMV + SpMTV + fused vector
updates + two device reductions).  Timed: exactly K iterations after W warm-up iterations,
bracketed by barrier + device synchronisation, max over ranks.  Also reported: a full solve
to tolerance (solve_time_s, solve_iters), the per-kernel roofline of the dominant kernel
(HIP-event timed), and the oracle's CPU LSQR on a bounded sample of iterations on this host.

N > 1 (torchrun): see DESIGN.md §Multi-GPU.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def log(*a):
    if int(os.environ.get('RANK', '0')) == 0:
        print(*a, file=sys.stderr, flush=True)


def build_system(config, device):
    import lssurf_amd as LS
    from lssurf_amd import synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    from lssurf_amd.smooth_fit import FitSystem
    t0 = time.time()
    D, kw = synthetic.points(config)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    t1 = time.time()
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, device=device)
    E_all = 1 / (1. / np.concatenate((S['Ed'], S['Ec'])))
    w = 1. / np.sqrt(E_all ** 2)
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.ones(w.size, bool))
    t2 = time.time()
    return fs, rhs, w, {'host_assembly_s': t1 - t0, 'device_formation_s': t2 - t1}


def cpu_baseline(fs, b_weighted, sample_iters, threads):
    """oracle/lsqr_cpu.c on the same formed A (downloaded from the device) and the same
    weighted rhs; a bounded sample of iterations, timed on this host's cores."""
    from oracle import cpu
    A = fs.solver.get_csr()
    x, st = cpu.lsqr(A, b_weighted, fixed_iters=sample_iters, threads=threads)
    return {'value': st['iters'] / st['time_s'], 'unit': 'LSQR iters/s', 'cores': int(st['threads']),
            'kind': 'port', 'sample': f'{int(st["iters"])} LSQR iterations of the same system (oracle/lsqr_cpu.c, '
                                      f'OpenMP, column-scaled), {st["time_s"]:.1f} s'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--config', default='c4')
    ap.add_argument('--no-solve', action='store_true', help='skip the full solve to tolerance')
    ap.add_argument('--cpu-iters', type=int, default=10)
    ap.add_argument('--no-cpu', action='store_true')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('gloo', init_method='env://')

    fs, rhs, w, setup = build_system(args.config, local)
    info = fs.solver.info()
    log(f'system: {info}, setup {setup}')

    def barrier():
        if dist is not None:
            dist.barrier()

    fs.solver.iterate(rhs, args.warmup)
    barrier()
    t0 = time.perf_counter()
    st = fs.solver.iterate(rhs, args.steps)   # synchronous: returns after the device finished
    barrier()
    t_wall = time.perf_counter() - t0
    t_dev = st['time_s']
    if dist is not None:
        import torch
        tt = torch.tensor([t_wall], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_wall = float(tt[0])

    ms_per_step = 1e3 * t_wall / args.steps
    value = world * args.steps / t_wall   # independent replicas
    Z, m, n = info['nnz'], info['m'], info['n']
    bytes_iter = st['bytes_per_iter']

    prof = fs.solver.profile_kernels(reps=10)
    # algorithmic bytes per launch (DESIGN.md §Byte model)
    kb = {'spmtv': 12.0 * Z + 8.0 * m + 16.0 * n, 'xw_spmv': 12.0 * Z + 16.0 * m + 48.0 * n}
    dom = max(('spmtv', 'xw_spmv'), key=lambda k: prof[k])
    achieved = kb[dom] / (prof[dom] * 1e-3) / 1e9

    solve = {}
    if not args.no_solve:
        x, sst = fs.solver.solve(rhs)
        solve = {'solve_time_s': sst['time_s'], 'solve_iters': int(sst['iters']), 'solve_istop': int(sst['istop'])}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = min(os.cpu_count() or 1, 16)
        cpu = cpu_baseline(fs, w * rhs, args.cpu_iters, threads)
    fs.close()

    if rank == 0:
        out = {
            'metric': 'LSQR iters/sec + solve wall-time, 1024x1024x12 grid / 2M pts, 1-8 GPU',
            'value': value, 'unit': 'LSQR iters/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': ms_per_step, 'higher_is_better': True,
            'scaling': 'weak' if world > 1 else 'strong', 'vs_baseline': None, 'dtype': 'f64',
            'data': 'synthetic (SURVEY.md §8(d) point cloud)',
            'config': {'workload': f'smooth_fit LSQR, {args.config}', 'grid': info, 'rows': m, 'cols': n,
                       'nnz': Z, 'precond': 'column scaling', 'mode': 'replicas' if world > 1 else 'single'},
            'device_iter_ms': 1e3 * t_dev / args.steps,
            'hbm_gbs_iter': bytes_iter * args.steps / t_dev / 1e9,
            'roofline': {'bound': 'hbm', 'kernel': dom, 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
                         'kernel_ms': prof},
            'cpu_baseline': cpu,
            **solve, **setup,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
