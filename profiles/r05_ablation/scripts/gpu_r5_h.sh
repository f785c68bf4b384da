#!/bin/bash
# round-5 GPU pass H: two-set loop schedule variant on the 128x128 layers; model forwards
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
timeout -k 10 400 ./tools/gemm_bench --reps 10 --shapes l3.convs0,l3.convs1,l2.conv1,l2.0.conv3,l3.0.conv3,fuse34.att0,l3_ds \
  $L ablibs/libspk_sch5.so ablibs/libspk_sch0.so > gpurun_out/r5_sched2.txt 2>&1 || exit $?
cat gpurun_out/r5_sched2.txt
for arch in eres2netv2 eres2net_large ecapa campplus; do
  timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/r5_steps_${arch}_h.json > gpurun_out/r5_steps_${arch}_h.txt 2>&1 || exit $?
  echo "$arch $(grep -v amdgpu.ids gpurun_out/r5_steps_${arch}_h.txt | head -1)"
done
