#!/bin/bash
# Variant build of libspk_hip.so for A/B runs (dev tool): one source compiled with extra
# flags, linked with the other in-tree objects into ablibs/libspk_<tag>.so (tools/gpu_ab.sh).
#   tools/variant_lib.sh <tag> <source.hip> [-DFLAG=...]
set -eu
cd "$(dirname "$0")/.."
tag=$1; src=$2; shift 2
make -s -j8 -C 3d-speaker_amd/csrc
base=$(basename "$src" .hip)
mkdir -p exp_libs/obj_$tag ablibs
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -w "$@" -c "$src" -o exp_libs/obj_$tag/$base.o
objs=$(ls 3d-speaker_amd/build/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ablibs/libspk_$tag.so $objs exp_libs/obj_$tag/$base.o \
    -L/opt/rocm/lib -lrocsolver -lrocblas
echo "built ablibs/libspk_$tag.so"
