#!/bin/bash
# tile-shape / stagger sweep of the LDS-DMA GEMM (dev tool): tools/gemm_bench under env arms
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r6e}
[ tools/gemm_bench -nt 3d-speaker_amd/csrc/common.h ] || { echo "gemm_bench older than common.h: rebuild it"; exit 2; }
for arm in ${ARMS:-default SPK_GEMM_F_TILE=128x128 SPK_GEMM_F_TILE=256x128 SPK_GEMM_F_TILE=128x256}; do
  echo "== $arm"
  if [ $arm = default ]; then e=""; else e="$arm"; fi
  env $e timeout -k 10 300 tools/gemm_bench --reps 20 --shapes ${SHAPES:-l3.conv1,l3.conv3,l4.conv1,l4.conv3,l4.convs0,l3.convs0,l3_ds} ${LIB:-ablibs/libspk_m16s.so} > gpurun_out/${TAG}_$arm.txt 2>&1 || exit $?
  grep -E " us " gpurun_out/${TAG}_$arm.txt | awk '{print $2}' | paste -sd' '
done
