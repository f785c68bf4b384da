#!/bin/bash
# round-5 GPU pass L: per-step profile of CAM++ / ECAPA with the scaled split (which kernels moved)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
timeout -k 10 300 ./tools/gemm_bench --reps 10 --shapes l3.conv1,l3.convs0,l4.convs0,l3_ds $L > gpurun_out/r5_scaled_gemm.txt 2>&1 || exit $?
cat gpurun_out/r5_scaled_gemm.txt
for arch in campplus ecapa; do
  timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/r5_steps_${arch}_l.json > gpurun_out/r5_steps_${arch}_l.txt 2>&1 || exit $?
  echo "$arch $(grep -v amdgpu.ids gpurun_out/r5_steps_${arch}_l.txt | head -1)"
done
