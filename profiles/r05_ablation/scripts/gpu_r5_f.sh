#!/bin/bash
# round-5 GPU pass F: S1 (K-concatenated shortcut) on the LDS-DMA GEMM, model timings, GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
for f in 0 1; do
  SPK_GEMM_F=$f timeout -k 10 300 ./tools/gemm_bench --reps 10 --shapes l2.0.conv3,l3.0.conv3,fuse34.att0 $L > gpurun_out/r5_s1_f$f.txt 2>&1 || exit $?
done
paste -d"\n" gpurun_out/r5_s1_f0.txt gpurun_out/r5_s1_f1.txt | awk "NR%2==1 || /us/"
for arch in eres2netv2 eres2net_large; do
  timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/r5_steps_${arch}_g.json > gpurun_out/r5_steps_${arch}_g.txt 2>&1 || exit $?
  echo "$arch $(grep -v amdgpu.ids gpurun_out/r5_steps_${arch}_g.txt | head -1)"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_gputest_f.log 2>&1; rc=$?; tail -3 gpurun_out/r5_gputest_f.log; exit $rc
