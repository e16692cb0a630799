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
ANISO = ('c5a', 'ta64', 'ta100')   # lssurf_amd.synthetic.ANISO (no package import before the PMC passes)


def log(*a):
    if int(os.environ.get('RANK', '0')) == 0:
        print(*a, file=sys.stderr, flush=True)


def _weights_rhs(S):
    """smooth_fit's first-iteration row weights 1/sqrt(E_all²) = |TCinv| (smooth_fit.py:103, 129;
    lssurf_amd.smooth_fit.iterate_fit) and right-hand side, host work before device formation."""
    w = np.abs(1. / np.concatenate((S['Ed'], S['Ec'])))
    rhs = np.zeros(w.size)
    rhs[:S['data'].size] = S['data'].z
    return w, rhs


def _runtime_start(device):
    """The process's one-time HIP start-up and code-object load (the first library handle,
    ≈ 0.1 s), kept off the device-formation clock: it is not formation of this system."""
    from lssurf_amd.solver import LSQSolver
    LSQSolver(device).close()


def build_system(config, device):
    import lssurf_amd as LS
    from lssurf_amd import synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    from lssurf_amd.smooth_fit import FitSystem
    _runtime_start(device)
    t0 = time.time()
    if config in synthetic.ANISO:   # BASELINE C5: the directional (anisotropic) z0 constraint
        S, kw = synthetic.aniso_system(config)
        t1 = time.time()
        fs = FitSystem(S['G_data'], S['Gc'], S['keep'], S['Gc'].col_N, device=device, grids=S['grids'])
        fs.solver.set_row_weight(S['w'])
        fs.solver.set_row_mask(np.ones(S['w'].size, bool))
        return fs, S['rhs'], S['w'], {'host_assembly_s': t1 - t0, 'device_formation_s': time.time() - t1}
    if config in synthetic.CONFIGS_2D:   # 2-D z0-only lin_op system (BASELINE C2), structured formation
        G, Gc, grid, w, rhs = synthetic.system2d(config)
        t1 = time.time()
        fs = FitSystem(G, Gc, np.arange(G.col_N), G.col_N, device=device, grids={'z0': grid})
        fs.solver.set_row_weight(w)
        fs.solver.set_row_mask(np.ones(w.size, bool))
        return fs, rhs, w, {'host_assembly_s': t1 - t0, 'device_formation_s': time.time() - t1}
    D, kw = synthetic.points(config)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    w, rhs = _weights_rhs(S)
    t1 = time.time()
    fs = FitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, device=device, grids=S['grids'])
    fs.solver.set_row_weight(w)
    fs.solver.set_row_mask(np.ones(w.size, bool))
    t2 = time.time()
    return fs, rhs, w, {'host_assembly_s': t1 - t0, 'device_formation_s': t2 - t1}


def build_dist_system(config, rank, world, device):
    """One rank of the y-slab distributed system (lssurf_amd.dist): every rank assembles the
    (lazy) operator description, generates only its own rows on its GPU and joins the RCCL
    communicator."""
    import lssurf_amd as LS
    from lssurf_amd import synthetic
    from lssurf_amd.constraint_functions import reference_epoch_keep_cols
    from lssurf_amd.dist import DistFitSystem
    t0 = time.time()
    D, kw = synthetic.points(config)
    S = LS.smooth_fit(data=D, return_fit_objects=True, VERBOSE=False, **kw)
    keep = reference_epoch_keep_cols(S['G_data'].col_N, S['grids']['dz'], kw['reference_epoch'])
    w, rhs = _weights_rhs(S)
    t1 = time.time()
    ds = DistFitSystem(S['G_data'], S['Gc'], keep, S['Gc'].col_N, rank, world, device)
    ds.iterate(w, rhs, 1)       # uploads weights / local rhs, builds the scaling and workspace
    t2 = time.time()
    return ds, rhs, w, {'host_assembly_s': t1 - t0, 'device_formation_s': t2 - t1}


class _Dist:
    """bench adapter: the same calls on a DistFitSystem rank as on an LSQSolver."""

    def __init__(self, ds):
        self.ds = ds

    def info(self):
        return self.ds.info()

    def iterate(self, rhs, iters, op=0, precond=1, method=0):
        return self.ds.iterate(None, None, iters, precond=precond, method=method)

    def solve(self, rhs, op=0, precond=1, method=0, b_rows=0):
        x = self.ds.solve(None, None, precond=precond, method=method)   # the single-GPU solve's tolerances
        return x, self.ds.stats

    def profile_cg(self, reps=10, precond=3):
        import ctypes
        o = np.zeros(8)
        rc = self.ds.L.lsq_profile_cg(self.ds.h, int(reps), int(precond), o.ctypes.data_as(ctypes.c_void_p))
        if rc != 0:
            raise RuntimeError('lsq_profile_cg: ' + self.ds.L.lsq_last_error(self.ds.h).decode())
        d = dict(zip(['cg_data', 'cg_normal', 'cg_update', 'cg_scalars'], o[:4].tolist()))
        d['bytes'] = {'cg_data': float(o[4]), 'cg_normal': float(o[5]), 'cg_update': float(o[6])}
        d['data_rows'] = 'matrix-free' if int(o[7]) & 1 else 'stored'
        d['normal_kernel'] = 'wave-strip' if int(o[7]) & 2 else 'ring'
        return d

    def profile_kernels(self, reps=10, op=0):
        import ctypes
        o = np.zeros(8)
        self.ds.L.lsq_profile_kernels(self.ds.h, int(reps), 0, o.ctypes.data_as(ctypes.c_void_p))
        d = dict(zip(['xw_spmv', 'spmtv', 'beta', 'givens'], o[:4].tolist()))
        d['bytes'] = {'xw_spmv': float(o[4]), 'spmtv': float(o[5])}
        return d


def host_cores():
    """The host cores this process may use ('all host cores, record nproc'):
    nproc (os.cpu_count), the affinity mask, the cgroup CPU quota (cpu.max: a container's share
    of a larger machine) and the socket count.  usable = min(affinity, ceil(quota))."""
    import math
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    for path in ('/sys/fs/cgroup/cpu.max', '/sys/fs/cgroup/cpu/cpu.cfs_quota_us'):
        try:
            parts = open(path).read().split()
        except OSError:
            continue
        if path.endswith('cpu.max') and parts and parts[0] != 'max':
            quota = float(parts[0]) / float(parts[1] if len(parts) > 1 else 100000)
        elif path.endswith('quota_us') and parts and int(parts[0]) > 0:
            period = float(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read().split()[0])
            quota = float(parts[0]) / period
        break
    sockets = set()
    for c in os.sched_getaffinity(0) if hasattr(os, 'sched_getaffinity') else range(nproc):
        try:
            sockets.add(open(f'/sys/devices/system/cpu/cpu{c}/topology/physical_package_id').read().strip())
        except OSError:
            pass
    usable = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return {'nproc': nproc, 'affinity': aff, 'cgroup_quota': quota, 'sockets': len(sockets) or None,
            'usable': usable}


def cpu_baseline(fs, w, b_weighted, sample_iters, threads, method=0, csr=True):
    """The same algorithm on this host's cores, on the same system and the same weighted rhs, a
    bounded sample of iterations: CGNR + block-Jacobi with the GPU solve's node blocks when the GPU
    line is CGNR — on the GPU's operator representation (oracle/cgnr_struct_cpu.c: stencil rows from
    the part descriptors, matrix-free data rows; `value`) and on the assembled CSR downloaded from the
    device (oracle/cgnr_cpu.c; `csr_port`) — else LSQR (oracle/lsqr_cpu.c)."""
    from oracle import cpu
    if method == 1 and getattr(fs, 'blocks', None) is not None:
        out = None
        if getattr(fs, 'desc', None) is not None:
            try:
                # half the CSR kind's sample: ~0.35 s per C4 iteration on 16 threads (two passes over
                # the 75 M rows and their weights, no stored matrix) against the CSR kind's ~0.14 s
                xs, st = cpu.cgnr_bj_struct(fs.desc, fs.n_full, w, fs.keep_cols, b_weighted, *fs.blocks,
                                            fixed_iters=max(10, sample_iters // 2), threads=threads)
                out = {'value': st['iters'] / st['time_s'], 'unit': 'CGNR iters/s', 'cores': int(st['threads']),
                       'kind': 'port', 'setup_s': st['setup_s'], 'operator': 'structured (matrix-free)',
                       'sample': f'{int(st["iters"])} CGNR + block-Jacobi iterations of the same system and node '
                                 f'blocks on the GPU line\'s operator representation (stencil rows from the part '
                                 f'descriptors, matrix-free data rows; oracle/cgnr_struct_cpu.c, OpenMP), '
                                 f'{st["time_s"]:.1f} s after {st["setup_s"]:.1f} s of point sort and block factors'}
            except ValueError as e:   # interpolation grids on different lattices: the CSR kind only
                log(f'bench: structured CPU baseline unavailable ({e})')
        if out is not None and not csr:
            return out
        A = fs.solver.get_csr()
        x, st = cpu.cgnr_bj(A, b_weighted, *fs.blocks, fixed_iters=sample_iters, threads=threads)
        csr = {'value': st['iters'] / st['time_s'], 'unit': 'CGNR iters/s', 'cores': int(st['threads']),
               'kind': 'port', 'setup_s': st['setup_s'], 'operator': 'assembled CSR',
               'sample': f'{int(st["iters"])} CGNR + block-Jacobi iterations of the same system and node blocks '
                         f'on the assembled CSR (oracle/cgnr_cpu.c, OpenMP), {st["time_s"]:.1f} s after '
                         f'{st["setup_s"]:.1f} s of transpose and block factors'}
        if out is None:
            return csr
        out['csr_port'] = csr
        return out
    A = fs.solver.get_csr()
    x, st = cpu.lsqr(A, b_weighted, fixed_iters=sample_iters, threads=threads)
    return {'value': st['iters'] / st['time_s'], 'unit': 'LSQR iters/s', 'cores': int(st['threads']),
            'kind': 'port', 'sample': f'{int(st["iters"])} LSQR iterations of the same system (oracle/lsqr_cpu.c, '
                                      f'OpenMP, column-scaled), {st["time_s"]:.1f} s'}


# kernel symbols per role: LSQR (assembled-SELL operator / structured stencil operator), CGNR
# (a role's launches per iteration: its PMC bytes are the sum over the symbols found)
KERNEL_SYMBOL = {0: {'xw_spmv': ('k_xw_spmv(', 'k_mf_fwd('), 'spmtv': ('k_spmtv(', 'k_mf_spmtv(')},
                 1: {'cg_data': ('k_cg_data(', 'k_cg_atdq(', 'k_cg_dmf_ad(', 'k_cg_ad_xedge<', 'k_cg_dmf_atq<'),
                     'cg_normal': ('k_cg_normal(', 'k_cg_normal_col<', 'k_cg_normal_col8(', 'k_cg_normal_rw<',
                                   'k_cg_xedge<'),
                     'cg_update': ('k_cg_block<', 'k_cg_jacobi(')}}


def pmc_traffic(config, op, method=0, precond=1, timeout=300):
    """HBM-side bytes per launch of each iteration kernel from rocprofv3 PMC counters, collected in two
    separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950) of a short
    child run of this script.  Units: KiB.  FETCH_SIZE is doubled: on gfx950 it reports exactly
    half the bytes of coalesced 4/8/16-B-per-lane streams (MI355X_MICROARCH.md §HBM; our own
    widths calibrated by profiles/calib_fetch.hip, profiles/r01_calib_fetch.md).  Counts
    Infinity-Cache hits too (the counters sit on the L2's fabric side).  Returns None (+ reason)
    when rocprofv3 is unavailable or fails.  Runs before this process touches the GPU."""
    import csv
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which('rocprofv3')
    if exe is None:
        return None, 'rocprofv3 not found'
    vals = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get('TMPDIR', '/tmp')) as tmp:
        for ctr in ('FETCH_SIZE', 'WRITE_SIZE'):
            out = os.path.join(tmp, ctr)
            cmd = [exe, '--pmc', ctr, '-d', out, '-o', 'run', '--output-format', 'csv', '--',
                   sys.executable, os.path.abspath(__file__), '--pmc-child', '--config', config, '--op', str(op),
                   '--method', ['lsqr', 'cgnr'][method], '--precond', str(precond)]
            try:
                r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=timeout,
                                   env=dict(os.environ, TMPDIR=tmp))
            except subprocess.TimeoutExpired:
                return None, f'rocprofv3 --pmc {ctr} timed out'
            if r.returncode != 0:
                return None, f'rocprofv3 --pmc {ctr} rc={r.returncode}'
            files = [os.path.join(dp, f) for dp, _, fs in os.walk(out) for f in fs if f.endswith('counter_collection.csv')]
            rows = [row for f in files for row in csv.DictReader(open(f)) if row['Counter_Name'] == ctr]
            for kernel, syms in KERNEL_SYMBOL[method].items():
                tot, found = 0.0, False
                for sym in syms:   # mean per launch of each symbol, summed over the role's symbols
                    xs = [float(r['Counter_Value']) for r in rows if sym in r['Kernel_Name']]
                    if xs:
                        tot += sum(xs) / len(xs)
                        found = True
                if not found:
                    return None, f'no {ctr} samples for {kernel}'
                vals[kernel, ctr] = tot * 1024.0
    return {k: {'fetch_bytes': 2.0 * vals[k, 'FETCH_SIZE'], 'write_bytes': vals[k, 'WRITE_SIZE'],
                'total': 2.0 * vals[k, 'FETCH_SIZE'] + vals[k, 'WRITE_SIZE']} for k in KERNEL_SYMBOL[method]}, None


def pmc_child(config, op, method, precond):
    """Short run under the profiler: formation + a few iterations of each kernel."""
    fs, rhs, w, _ = build_system(config, 0)
    fs.solver.iterate(rhs, 4, op=op, method=method, precond=precond)
    fs.close()


def e2e(config, iters):
    """smooth_fit end to end (host assembly, device formation, editing loop, outputs) with the
    library defaults; prints its timing breakdown as one JSON line."""
    import lssurf_amd as LS
    from lssurf_amd import synthetic
    D, kw = synthetic.points(config)
    t0 = time.time()
    S = LS.smooth_fit(data=D, VERBOSE=False, max_iterations=iters, **kw)
    wall = time.time() - t0
    tim = {k: (v if not isinstance(v, dict) else {kk: vv for kk, vv in v.items() if kk in ('iters', 'istop', 'time_s')})
           for k, v in S['timing'].items()}
    print(json.dumps({'config': config, 'max_iterations': iters, 'wall_s': wall, 'timing': tim,
                      'n_edited': int(np.sum(S['data'].three_sigma_edit == 0))}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--config', default='c4')
    ap.add_argument('--no-solve', action='store_true', help='skip the full solve to tolerance')
    ap.add_argument('--cpu-iters', type=int, default=80,
                    help='iterations of the CPU baseline sample (the GPU line\'s algorithm: CGNR + block-Jacobi, or LSQR)')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--cpu-solve', action='store_true',
                    help='also run the CPU oracle LSQR to the solve tolerance (BASELINE.md §4 parity at size; slow)')
    ap.add_argument('--dist', action='store_true', help='use the distributed (RCCL) path even at N=1')
    ap.add_argument('--no-pmc', action='store_true', help='skip the rocprofv3 PMC traffic passes')
    ap.add_argument('--op', type=int, default=0, help='0: auto (structured stencil operator), 1: assembled SELL')
    ap.add_argument('--same-device', action='store_true',
                    help='testing only: every rank on device 0 (RCCL over loopback sockets, distinct host ids)')
    ap.add_argument('--precond', type=int, default=3,
                    help='1: column scaling, 3: block-Jacobi per (y,x) node (smooth_fit default at this size)')
    ap.add_argument('--solve-precond', default='auto', choices=['auto', '1', '3', '4'],
                    help='preconditioner of the full solve: auto = multigrid (4) where it runs, else --precond')
    ap.add_argument('--method', default='cgnr', choices=['cgnr', 'lsqr'],
                    help='cgnr: PCG on the normal equations, fused normal-stencil operator (smooth_fit default); '
                         'lsqr: LSQR on the stencil operator')
    ap.add_argument('--pmc-child', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--e2e', type=int, default=0, metavar='ITERS',
                    help='instead of the bench line: time smooth_fit end to end with max_iterations=ITERS')
    args = ap.parse_args()
    if args.e2e:
        return e2e(args.config, args.e2e)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if (world > 1 or args.dist) and args.method == 'lsqr':   # distributed LSQR: column scaling only
        args.precond = 1
    if args.config in __import__('lssurf_amd.synthetic', fromlist=['x']).CONFIGS_2D:
        if world > 1 or args.dist:
            raise SystemExit('bench: the 2-D configs run on one GPU')
        args.precond = 1   # no node blocks in a z0-only system: Jacobi
    meth = 1 if args.method == 'cgnr' else 0
    if args.pmc_child:
        return pmc_child(args.config, args.op, meth, args.precond)
    pmc, pmc_note = None, 'skipped (--no-pmc, --dist or N>1)'
    if world == 1 and not args.no_pmc and not args.dist:
        pmc, pmc_note = pmc_traffic(args.config, args.op, meth, args.precond)   # child processes, before this one touches the GPU

    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch.distributed as dist
        from lssurf_amd.dist import _quiet_stdout   # gloo announces its peers on stdout
        _quiet_stdout(lambda: dist.init_process_group('gloo', init_method='env://'))

    if args.same_device:   # RCCL refuses two ranks on one device of one host
        os.environ['NCCL_HOSTID'] = f'lsq-bench-host-{rank}'
        os.environ.setdefault('NCCL_SOCKET_IFNAME', 'lo')
        os.environ.setdefault('NCCL_IB_DISABLE', '1')
        local = 0
    if world > 1 or args.dist:
        ds, rhs, w, setup = build_dist_system(args.config, rank, world, local)
        solver = _Dist(ds)
        fs = ds
    else:
        fs, rhs, w, setup = build_system(args.config, local)
        solver = fs.solver
    info = solver.info()
    log(f'system: {info}, setup {setup}')

    def barrier():
        if dist is not None:
            dist.barrier()

    def gather(obj):   # every rank's object, in rank order (gloo; set-up / reporting only)
        if dist is None:
            return [obj]
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    ranks = None
    if world > 1 or args.dist:
        # self-check of a multi-GPU run: what each rank's RCCL communicator and device
        # report; the run fails unless RCCL sees all N ranks and (without --same-device) every rank
        # drives a card of its own
        ranks = gather(dict(fs.comm_info(), rank=rank))
        bad = [r for r in ranks if r['comm_count'] != world]
        cards = [r['pci'] for r in ranks]
        if bad or (not args.same_device and len(set(cards)) != len(cards)):
            log(f'bench: multi-GPU self-check failed: {ranks}')
            raise SystemExit(3)

    solver.iterate(rhs, args.warmup, op=args.op, precond=args.precond, method=meth)
    barrier()
    t0 = time.perf_counter()
    st = solver.iterate(rhs, args.steps, op=args.op, precond=args.precond, method=meth)   # synchronous: returns after the device finished
    barrier()
    t_wall = time.perf_counter() - t0
    t_dev = st['time_s']
    if dist is not None:
        import torch
        tt = torch.tensor([t_wall], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_wall = float(tt[0])

    if ranks is not None:   # per-rank device time of the timed iterations
        for r, t in zip(ranks, gather(1e3 * st['time_s'] / args.steps)):
            r['iter_ms_device'] = t
    ms_per_step = 1e3 * t_wall / args.steps
    value = args.steps / t_wall   # LSQR iterations of the ONE (row-partitioned) system per second
    Z, m, n = info['nnz'], info['m'], info['n']      # this rank's (local) system
    gm, gZ, gn = m, Z, n
    if dist is not None:                              # whole-system sizes for the config record
        import torch
        tt = torch.tensor([m, Z], dtype=torch.int64)
        dist.all_reduce(tt)
        gm, gZ = int(tt[0]), int(tt[1])
    if isinstance(solver, _Dist):
        gn = int(fs.keep_cols.size)
    bytes_iter = st['bytes_per_iter']

    if meth == 1:
        prof = solver.profile_cg(reps=10, precond=args.precond)
        roles = ('cg_data', 'cg_normal', 'cg_update')
    else:
        prof = solver.profile_kernels(reps=10, op=args.op)
        roles = ('spmtv', 'xw_spmv')
    # algorithmic bytes per launch (DESIGN.md §Byte model)
    kb = prof.pop('bytes')   # algorithmic bytes per launch, from the library's byte model
    data_rows = prof.pop('data_rows', None)   # CGNR: 'matrix-free' (points sorted by cell) or 'stored'
    normal_kernel = prof.pop('normal_kernel', None)   # CGNR: 'wave-strip' (k_cg_normal_rw) or 'ring'
    dom = max(roles, key=lambda k: prof[k])
    achieved = kb[dom] / (prof[dom] * 1e-3) / 1e9

    solve = {}
    if not args.no_solve:
        # solve wall-time with smooth_fit's default solver for this system: CGNR + the multigrid
        # V-cycle (precond 4) where it runs (per-node blocks; over ranks: window level 0 + the
        # replicated global coarse levels), else the timed configuration; then CGNR + block-Jacobi
        # and (one GPU) LSQR + block-Jacobi for comparison
        names = {1: 'column scaling', 3: 'block-Jacobi per (y,x) node', 4: 'multigrid V-cycle (block-Jacobi smoothing)'}
        sp = args.precond
        nzr = np.flatnonzero(rhs)   # b[b_rows:] == 0 (the constraint rows): only b[:b_rows] is uploaded
        b_rows = int(nzr[-1]) + 1 if nzr.size else 0
        mg_ok = (getattr(fs, 'has_global', False) and fs.has_blocks) if isinstance(solver, _Dist) \
            else solver.cg_available(4)[0]
        if (args.solve_precond == 'auto' and meth == 1 and args.precond == 3 and mg_ok) or args.solve_precond == '4':
            sp = 4

        def rec(st):
            # solve_time_s: device iterations; solve_setup_s: the per-solve preconditioner set-up
            # (block factors / multigrid levels, λ estimates) that every solve pays; total = both
            return {'solve_time_s': st['time_s'], 'solve_setup_s': st.get('setup_s', 0.0),
                    'solve_total_s': st['time_s'] + st.get('setup_s', 0.0),
                    'solve_iters': int(st['iters']), 'solve_istop': int(st['istop']),
                    'solve_comm_bytes_per_iter': float(st.get('comm_bytes_per_iter', 0.0)),
                    'solve_iters_per_s': st['iters'] / st['time_s'] if st['time_s'] > 0 else None,
                    'solve_roofline': {'bytes_per_iter': st['bytes_per_iter'],
                                       'achieved_gbs': st['bytes_per_iter'] * st['iters'] / st['time_s'] / 1e9
                                       if st['time_s'] > 0 else None,
                                       'frac': st['bytes_per_iter'] * st['iters'] / st['time_s'] / 1e9 / HBM_PEAK_GBS
                                       if st['time_s'] > 0 else None}}
        # an untimed first solve: its set-up also captures and instantiates the iteration's hipGraph
        # (host work once per system and preconditioner — smooth_fit's later outer iterations
        # replay it); the timed solve's set-up is what every solve pays (factors, λ, first V-cycle)
        if os.environ.get('LSQ_BENCH_MAPS'):   # development: library load addresses for a host crash stack
            with open('/proc/self/maps') as f, open(os.environ['LSQ_BENCH_MAPS'], 'w') as g:
                g.write(f.read())
        x1, sfirst = solver.solve(rhs, op=args.op, precond=sp, method=meth, b_rows=b_rows)
        x, sst = solver.solve(rhs, op=args.op, precond=sp, method=meth, b_rows=b_rows)
        solve = dict(rec(sst), solve_method=['lsqr', 'cgnr'][int(sst.get('method', 0))],
                     solve_precond=names.get(sp, sp), solve_setup_first_s=sfirst.get('setup_s', 0.0),
                     solve_iters_first=int(sfirst['iters']),
                     solve_rel_diff_first=float(np.linalg.norm(x - x1) / max(np.linalg.norm(x), 1e-300)))
        if meth == 1 and sp == 4:
            xb, sb = solver.solve(rhs, op=args.op, precond=3, method=1, b_rows=b_rows)
            solve['solve_block_jacobi'] = rec(sb)
            solve['solve_rel_diff_vs_block_jacobi'] = float(np.linalg.norm(x - xb) / np.linalg.norm(xb))
        if meth == 1 and not isinstance(solver, _Dist):   # distributed LSQR has no block-Jacobi
            xl, sl = solver.solve(rhs, op=args.op, precond=min(args.precond, 3), method=0, b_rows=b_rows)
            solve['solve_lsqr'] = rec(sl)
            solve['lsqr_iters_per_s'] = solve['solve_lsqr']['solve_iters_per_s']
            solve['solve_rel_diff_vs_lsqr'] = float(np.linalg.norm(x - xl) / np.linalg.norm(xl))

    if ranks is not None and solve:   # per-rank bytes sent per iteration of the full solve
        for r, b in zip(ranks, gather(solve['solve_comm_bytes_per_iter'])):
            r['solve_comm_bytes_per_iter'] = b
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and not args.dist:
        hc = host_cores()
        threads = hc['usable']   # every core this process may use, one OpenMP thread per core, pinned
        os.environ.setdefault('OMP_PROC_BIND', 'close')   # read by libgomp when oracle/_cpu.so loads
        os.environ.setdefault('OMP_PLACES', 'cores')
        cpu = cpu_baseline(fs, w, w * rhs, args.cpu_iters, threads, meth)
        cpu['host'] = hc
        if threads != 16 and os.environ.get('LSQ_BENCH_CPU16', '1') != '0' and meth == 1 \
                and getattr(fs, 'desc', None) is not None:
            # rounds 4-5 reported 16 threads: kept beside the all-cores figure for continuity
            try:
                c16 = cpu_baseline(fs, w, w * rhs, args.cpu_iters, 16, meth, csr=False)
                cpu['threads16'] = {k: c16[k] for k in ('value', 'unit', 'cores')}
            except Exception as e:   # noqa: BLE001 - reporting only
                log(f'bench: 16-thread CPU baseline failed ({e})')
        if args.cpu_solve and solve:   # the CPU oracle to the same stopping rule, on the same A, b
            from oracle import cpu as ocpu
            xc, stc = ocpu.lsqr(fs.solver.get_csr(), w * rhs, atol=1e-10, btol=1e-10, conlim=1e8,
                                maxit=50 * int(info['n']), threads=threads)
            cpu.update({'solve_time_s': stc['time_s'], 'solve_iters': int(stc['iters']),
                        'solve_istop': int(stc.get('istop', -1)),
                        'solve_rule': 'LSQR, column scaling, atol = btol = 1e-10 (the GPU solves\' rule)',
                        'solve_rel_diff_gpu_vs_cpu': float(np.linalg.norm(x - xc) / np.linalg.norm(xc))})
    fs.close()

    traffic, traffic_note = (pmc[dom]['total'], pmc) if pmc else (None, pmc_note)
    method_name = {0: 'LSQR', 1: 'CGNR (PCG on AᵀA)'}[int(st.get('method', meth))]

    if rank == 0:
        out = {
            'metric': 'LSQR iters/sec + solve wall-time, 1024x1024x12 grid / 2M pts, 1-8 GPU',
            'value': value, 'unit': 'CGNR iters/s (block-Jacobi PCG on AᵀA = LSQR\'s iterates on A·M^-1/2)'
                                    if meth == 1 else 'LSQR iters/s',
            'solver': method_name, 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': ms_per_step, 'higher_is_better': True,
            'scaling': 'strong', 'vs_baseline': None, 'dtype': 'f64',
            'data': 'synthetic (SURVEY.md §8(d) point cloud)',
            'config': {'workload': f'{"2-D lin_op (z0 only)" if args.config in ("c2", "t2d") else "smooth_fit"} solve, {args.config}'
                                   + (' (directional z0 constraint, aniso notebook)' if args.config in ANISO else ''),
                       'rank0_system': info, 'rows': gm, 'cols': gn,
                       'nnz': gZ, 'precond': {1: 'column scaling', 3: 'block-Jacobi per (y,x) node'}.get(args.precond, args.precond),
                       'operator': ('structured stencil rows + ' + ('matrix-free data rows (points sorted by cell)'
                                                                     if data_rows == 'matrix-free' else 'SELL data rows'))
                       if (fs.structured if isinstance(solver, _Dist) else info.get('stencil_op') and args.op == 0)
                       else 'assembled SELL',
                       'normal_kernel': normal_kernel,
                       'parallelism': f'y-slab rows x{world} (RCCL)' if world > 1 or args.dist else 'single'},
            'device_iter_ms': 1e3 * t_dev / args.steps,
            'hbm_gbs_iter': bytes_iter * args.steps / t_dev / 1e9,
            'roofline': {'bound': 'hbm', 'kernel': dom, 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'algorithmic_bytes': kb[dom], 'traffic_detail': traffic_note, 'kernel_ms': prof},
            'cpu_baseline': cpu,
            **solve, **setup,
        }
        if ranks is not None:
            its = [r['iter_ms_device'] for r in ranks]
            out['ranks'] = ranks
            out['rank_iter_ms_device'] = {'max': max(its), 'min': min(its)}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
