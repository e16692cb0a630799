# Build a variant of liblsqsurf.so whose band.hip gets extra compile flags (A/B of the band
# kernels):  bash tools/build_band_variant.sh <name> [-DFLAG ...]  →  tools/ab/lib_<name>.so
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
python -m lssurf_amd.build > /dev/null
mkdir -p tools/ab /tmp/abobj
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-result "$@" \
    -c lssurf_amd/csrc/band.hip -o /tmp/abobj/band_$name.o
objs=""
for s in scan build assemble dense lsqr block api tri rde; do objs="$objs lssurf_amd/csrc/build/$s.o"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/ab/lib_$name.so $objs /tmp/abobj/band_$name.o \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo tools/ab/lib_$name.so
