#!/bin/bash
# round-5 GPU pass B: LDS-DMA GEMM tile sweep against the register-staged kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
SPK_GEMM_F=0 timeout -k 10 200 ./tools/gemm_bench --reps 10 $L > gpurun_out/r5_tile_old.txt 2>&1 || exit $?
for t in 128x128 256x128 128x256 256x256; do
  SPK_GEMM_F_TILE=$t timeout -k 10 200 ./tools/gemm_bench --reps 10 $L > gpurun_out/r5_tile_$t.txt 2>&1 || exit $?
  echo "tile $t done"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3_full.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/r5_c3_full.log 2>&1; rc=$?; tail -25 gpurun_out/r5_c3_full.log; exit $rc
