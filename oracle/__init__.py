"""oracle/ — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference's algorithms on LSsurf's solve path, used solely as the
checker by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg.
Nothing in ``lssurf_amd`` imports, links or executes anything in this directory; the product
path fails loudly when its HIP library is missing instead of falling back here.

Contents
--------
dense.py        exact least squares (stand-in for SuiteSparseQR ``sparseqr.solve`` / ``rz``,
                PySPQR, unpinned version — not vendored in /root/reference)
lsqr_cpu.c      C/OpenMP restatement of Paige–Saunders LSQR (scipy.sparse.linalg.lsqr stop
                rules) on CSR — the CPU baseline ("port") and large-size parity checker
tri_upper.c     C restatement of the three Cython triangular kernels
                (LSsurf/inv_tr_upper.pyx:19-94, propagate_qz_errors.pyx:15-69,
                spsolve_tr_upper.pyx:11-54)
cpu.py          ctypes loader for the two C files above (built into oracle/_cpu.so)
build_ref.sh    compiles the reference's own .pyx kernels into oracle/_ref/ (the pin for
                tri_upper.c and for lssurf_amd's tri kernels)
"""
