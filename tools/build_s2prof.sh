#!/bin/bash
# Diagnostic build of libspk_hip.so with the fused stage-2 block's phase stamps
# (-DSPK_S2_PROF=1, ablation -DSPK_S2_EXP=$e for each e in EXPS) into ab/libspk_s2prof$e.so (tools/s2_prof.py reads them).
set -eu
cd "$(dirname "$0")/.."
make -s -j8 -C 3d-speaker_amd/csrc
mkdir -p exp_libs/obj_s2prof ab
objs=$(ls 3d-speaker_amd/build/*.o | grep -v res2block_s2)
for e in ${EXPS:-0}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSPK_S2_PROF=1 -DSPK_S2_EXP=$e \
      -c 3d-speaker_amd/csrc/res2block_s2.hip -o exp_libs/obj_s2prof/res2block_s2_$e.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ab/libspk_s2prof$e.so $objs exp_libs/obj_s2prof/res2block_s2_$e.o \
      -L/opt/rocm/lib -lrocsolver -lrocblas
done
