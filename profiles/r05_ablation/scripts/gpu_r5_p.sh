#!/bin/bash
# round-5 GPU pass P: 256x256 direct epilogue (accumulators straight to memory) vs the LDS rows
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
timeout -k 10 400 ./tools/gemm_bench --reps 20 --shapes l3.conv1,l3.conv3,l4.conv1,l4.conv3,l4.convs0,l3_ds,ec.tdnn1 \
  ablibs/libspk_nodirect.so $L > gpurun_out/r5_direct_ab.txt 2>&1 || { cat gpurun_out/r5_direct_ab.txt; exit 1; }
cat gpurun_out/r5_direct_ab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_c2_full.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_direct_tests.log 2>&1 || { tail -30 gpurun_out/r5_direct_tests.log; exit 1; }
tail -1 gpurun_out/r5_direct_tests.log
for i in 1 2; do
  timeout -k 10 300 python tools/profile_steps.py --arch eres2netv2 > gpurun_out/r5_steps_direct$i.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r5_steps_direct$i.txt | head -1
done
