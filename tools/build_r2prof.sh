#!/bin/bash
# Diagnostic build of libspk_hip.so with the fused Res2Net block's phase stamps
# (-DSPK_R2_PROF=1) into exp_libs/libspk_r2prof.so (tools/r2_prof.py reads them).
set -eu
cd "$(dirname "$0")/.."
make -s -j8 -C 3d-speaker_amd/csrc
mkdir -p exp_libs/obj_r2prof
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSPK_R2_PROF=1 -c 3d-speaker_amd/csrc/res2block.hip \
    -o exp_libs/obj_r2prof/res2block.o
objs=$(ls 3d-speaker_amd/build/*.o | grep -v '/res2block.o')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o exp_libs/libspk_r2prof.so $objs exp_libs/obj_r2prof/res2block.o \
    -L/opt/rocm/lib -lrocsolver -lrocblas
