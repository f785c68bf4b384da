#!/bin/bash
# round-5 GPU pass J: 256x128 / 128x256 tiles with the one-set loop on the 104 / 208-wide layers
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
for t in 128x128 256x128 128x256 256x256; do
  SPK_GEMM_F_TILE=$t timeout -k 10 300 ./tools/gemm_bench --reps 10 --shapes l3.convs0,l3.convs1,l2.conv1,l3.conv1,l4.convs0,l3.conv3 $L > gpurun_out/r5_tilej_$t.txt 2>&1 || exit $?
done
