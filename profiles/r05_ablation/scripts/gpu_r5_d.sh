#!/bin/bash
# round-5 GPU pass D: GEMM shapes + per-model forward, LDS-DMA GEMM on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
timeout -k 10 300 ./tools/gemm_bench --reps 10 $L > gpurun_out/r5_gemm_d.txt 2>&1 || exit $?
for arch in eres2netv2 eres2net_large ecapa campplus; do
  for f in 1 0; do
    SPK_GEMM_F=$f timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/r5_steps_${arch}_f$f.json > gpurun_out/r5_steps_${arch}_f$f.txt 2>&1 || exit $?
    echo "$arch F=$f $(grep -v amdgpu.ids gpurun_out/r5_steps_${arch}_f$f.txt | head -1)"
  done
done
