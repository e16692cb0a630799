"""Build liblsqsurf.so (gfx950) in-tree with hipcc; no JIT cache, the .so travels with the repo.

Usage: python -m lssurf_amd.build [--force]
"""
import os
import subprocess
import sys
import concurrent.futures as cf

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
OBJ = os.path.join(CSRC, 'build')
LIB = os.path.join(HERE, 'liblsqsurf.so')
ARCH = 'gfx950'
SOURCES = ['scan.hip', 'build.hip', 'assemble.hip', 'lsqr.hip', 'dense.hip', 'band.hip', 'block.hip', 'api.hip', 'tri.hip', 'rde.hip']
# bit-exact recurrences (triangular kernels, formation) must not be FMA-contracted
NO_CONTRACT = {'tri.hip', 'build.hip', 'assemble.hip', 'rde.hip'}
COMMON = ['-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-Wall', '-Wno-unused-function',
          '-Wno-unused-result']


def _hipcc():
    for p in [os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc']:
        if p and os.path.exists(p):
            return p
    return 'hipcc'


def _deps_newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(('.hpp', '.inc'))]
    headers.append(os.path.join(os.path.dirname(HERE), 'include', 'lsqsurf.h'))
    jobs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src.replace('.hip', '.o'))
        if force or _deps_newer(o, [s] + headers):
            flags = COMMON + (['-ffp-contract=off'] if src in NO_CONTRACT else [])
            jobs.append([_hipcc(), *flags, '-c', s, '-o', o])
    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose and (r.stdout or r.stderr):
            print(r.stdout, r.stderr)
    with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 8) or 1) as ex:
        list(ex.map(run, jobs))
    objs = [os.path.join(OBJ, s.replace('.hip', '.o')) for s in SOURCES]
    if force or jobs or not os.path.exists(LIB):
        run([_hipcc(), '-shared', f'--offload-arch={ARCH}', '-o', LIB, *objs, '-L/opt/rocm/lib', '-lrccl',
             '-Wl,-rpath,/opt/rocm/lib'])
    return LIB


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
