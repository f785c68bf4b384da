#!/bin/bash
# round-5 GPU pass A: GEMM ablations of the LDS-DMA kernel, the GPU test suite, ERes2NetV2 steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 ./tools/gemm_bench --reps 10 --shapes l3.conv1,l3.conv3,l3.convs0,l4.convs0,l3_ds \
  3d-speaker_amd/lib/libspk_hip.so ablibs/libspk_f1.so ablibs/libspk_f2.so ablibs/libspk_f4.so ablibs/libspk_f6.so \
  ablibs/libspk_f8.so ablibs/libspk_f16.so ablibs/libspk_f31.so > gpurun_out/r5_fexp.txt 2>&1 || exit $?
echo "ablations done"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_gputest_a.log 2>&1 || { tail -30 gpurun_out/r5_gputest_a.log; exit 1; }
tail -3 gpurun_out/r5_gputest_a.log
timeout -k 10 300 python tools/profile_steps.py --arch eres2netv2 --json gpurun_out/r5_steps_v2_a.json > gpurun_out/r5_steps_v2_a.txt 2>&1 || exit $?
head -1 gpurun_out/r5_steps_v2_a.txt
