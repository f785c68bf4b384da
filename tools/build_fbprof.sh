#!/bin/bash
# Diagnostic build of libspk_hip.so with the Fbank frames kernel phase stamps
# (-DSPK_FB_PROF=1) into exp_libs/libspk_fbprof.so (tools/fb_prof.py reads them).
set -eu
cd "$(dirname "$0")/.."
make -s -j8 -C 3d-speaker_amd/csrc
mkdir -p exp_libs/obj_fbprof
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSPK_FB_PROF=1 ${FB_EXTRA:-} -c 3d-speaker_amd/csrc/fbank.hip \
    -o exp_libs/obj_fbprof/fbank.o
objs=$(ls 3d-speaker_amd/build/*.o | grep -v '/fbank.o')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o exp_libs/libspk_fbprof.so $objs exp_libs/obj_fbprof/fbank.o \
    -L/opt/rocm/lib -lrocsolver -lrocblas
