#!/bin/bash
# Ablation builds of the LDS-DMA ring GEMM (conv_gemm_ring.hip, -DSPK_REXP=N) linked with the
# in-tree objects into exp_libs/libspk_rN.so (dev tool; A/B with tools/gpu_ab.sh).
#   1 no MFMA   2 no in-loop DMA   3 no epilogue stores   4 no operand split   5 = 1+2+3   6 empty
set -eu
cd "$(dirname "$0")/.."
make -s -j8 -C 3d-speaker_amd/csrc
objs=$(ls 3d-speaker_amd/build/*.o | grep -v '/conv_gemm_ring.o')
for n in ${REXPS:-1 2 3 4}; do
  (
    mkdir -p exp_libs/obj_r$n
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -w -DSPK_REXP=$n -c 3d-speaker_amd/csrc/conv_gemm_ring.hip \
        -o exp_libs/obj_r$n/conv_gemm_ring.o
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o exp_libs/libspk_r$n.so $objs exp_libs/obj_r$n/conv_gemm_ring.o \
        -L/opt/rocm/lib -lrocsolver -lrocblas
    echo "built exp_libs/libspk_r$n.so"
  ) &
done
wait
