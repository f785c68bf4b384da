#!/bin/bash
# Ablation builds of the tiled conv GEMM (conv_gemm.hip, -DSPK_GEXP=N) linked with the
# in-tree objects into exp_libs/libspk_gN.so (dev tool; A/B with tools/gpu_ab.sh).
#   1 no MFMA   2 no operand split   3 no in-loop global loads
#   5 no in-loop LDS stores
set -eu
cd "$(dirname "$0")/.."
make -s -j8 -C 3d-speaker_amd/csrc
objs=$(ls 3d-speaker_amd/build/*.o | grep -v '/conv_gemm.o')
for n in ${GEXPS:-1 2 3 5}; do
  (
    mkdir -p exp_libs/obj_g$n
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -w -DSPK_GEXP=$n -c 3d-speaker_amd/csrc/conv_gemm.hip \
        -o exp_libs/obj_g$n/conv_gemm.o
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o exp_libs/libspk_g$n.so $objs exp_libs/obj_g$n/conv_gemm.o \
        -L/opt/rocm/lib -lrocsolver -lrocblas
    echo "built exp_libs/libspk_g$n.so"
  ) &
done
wait
