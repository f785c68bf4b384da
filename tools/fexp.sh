#!/bin/bash
# Ablation builds of the LDS-DMA conv GEMM (conv_gemm_f.hip, -DSPK_FEXP=N, bit mask) linked
# with the in-tree objects into ablibs/libspk_fN.so (dev tool; time them with tools/gemm_bench).
set -eu
cd "$(dirname "$0")/.."
make -s -j8 -C 3d-speaker_amd/csrc
objs=$(ls 3d-speaker_amd/build/*.o | grep -v '/conv_gemm_f.o')
for n in ${FEXPS:-1 2 4 8 16}; do
  (
    mkdir -p exp_libs/obj_f$n
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -w -DSPK_FEXP=$n -c 3d-speaker_amd/csrc/conv_gemm_f.hip \
        -o exp_libs/obj_f$n/conv_gemm_f.o
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ablibs/libspk_f$n.so $objs exp_libs/obj_f$n/conv_gemm_f.o \
        -L/opt/rocm/lib -lrocsolver -lrocblas
    echo "built ablibs/libspk_f$n.so"
  ) &
done
wait
