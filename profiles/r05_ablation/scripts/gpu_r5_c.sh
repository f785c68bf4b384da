#!/bin/bash
# round-5 GPU pass C: per-model forward with and without the LDS-DMA GEMM, 256x256 ablations,
# golden tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
timeout -k 10 300 ./tools/gemm_bench --reps 10 --shapes l3.conv1,l4.convs0,l3_ds,l4.conv3 $L ablibs/libspk_f1.so \
  ablibs/libspk_f6.so ablibs/libspk_f8.so ablibs/libspk_f16.so ablibs/libspk_f31.so > gpurun_out/r5_fexp256.txt 2>&1 || exit $?
echo ablations done
for arch in eres2netv2 eres2net_large ecapa campplus; do
  for f in 1 0; do
    SPK_GEMM_F=$f timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/r5_steps_${arch}_f$f.json > gpurun_out/r5_steps_${arch}_f$f.txt 2>&1 || exit $?
    echo "$arch F=$f $(grep -v amdgpu.ids gpurun_out/r5_steps_${arch}_f$f.txt | head -1)"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_c2_full.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_gputest_c.log 2>&1; rc=$?; tail -3 gpurun_out/r5_gputest_c.log; exit $rc
