# Build a variant of liblsqsurf.so with extra compile flags for the A/B harness (tools/ab_lib.sh):
#   bash tools/build_variant.sh <name> [-DFLAG ...]  →  tools/ab/lib_<name>.so
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
python -m lssurf_amd.build > /dev/null
mkdir -p tools/ab /tmp/abobj
for s in lsqr block; do   # the sources that hold the kernels under study (flags: -D switches)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-result "$@" \
      -c lssurf_amd/csrc/$s.hip -o /tmp/abobj/${s}_$name.o &
done
wait
objs=""
for s in scan build assemble dense band api tri rde; do objs="$objs lssurf_amd/csrc/build/$s.o"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/ab/lib_$name.so $objs /tmp/abobj/lsqr_$name.o /tmp/abobj/block_$name.o \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo tools/ab/lib_$name.so
