#!/usr/bin/env bash
# Build the reference's own Cython triangular kernels from their sources where they lie
# (/root/reference/LSsurf/{inv_tr_upper,propagate_qz_errors,spsolve_tr_upper}.pyx, built by the
# reference's setup.py:56-60) into oracle/_ref/.  Test infrastructure only: the outputs are the
# checker for lssurf_amd's tri_upper_* kernels and are never imported by the product path.
# No-op when /root/reference is absent (the GPU box uses the prebuilt files).
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
src=/root/reference/LSsurf
out="$here/_ref"
[ -d "$src" ] || { echo "build_ref: $src absent, keeping prebuilt oracle/_ref"; exit 0; }
mkdir -p "$out"
py=${PYTHON:-python3}
inc_py=$($py -c "import sysconfig;print(sysconfig.get_paths()['include'])")
inc_np=$($py -c "import numpy;print(numpy.get_include())")
suf=$($py -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
for k in inv_tr_upper propagate_qz_errors spsolve_tr_upper; do
  if [ ! -f "$out/$k$suf" ] || [ "$src/$k.pyx" -nt "$out/$k$suf" ]; then
    cython -3 -o "$out/$k.c" "$src/$k.pyx"
    gcc -shared -fPIC -O2 -w -I"$inc_py" -I"$inc_np" -DNPY_NO_DEPRECATED_API=NPY_1_7_API_VERSION \
        -o "$out/$k$suf" "$out/$k.c"
    rm -f "$out/$k.c"   # the generated C is an intermediate: only the built module is kept
  fi
done
echo "build_ref: built $(ls "$out"/*"$suf" | wc -l) reference kernels into $out"
