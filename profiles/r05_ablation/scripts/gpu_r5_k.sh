#!/bin/bash
# round-5 GPU pass K: scaled split (ECAPA / CAM++ without the exact twin): range-guard and model
# tests, GEMM regression check, model forwards scaled vs twin, per-step profiles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_range_guard.py tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_scaled_tests.log 2>&1 || { tail -40 gpurun_out/r5_scaled_tests.log; exit 1; }
tail -2 gpurun_out/r5_scaled_tests.log
timeout -k 10 300 ./tools/gemm_bench --reps 10 --shapes l3.conv1,l3.convs0,l4.convs0,l3_ds $L > gpurun_out/r5_scaled_gemm.txt 2>&1 || exit $?
cat gpurun_out/r5_scaled_gemm.txt
for mode in scaled twin; do
  SPK_RANGE_MODE=$mode timeout -k 10 400 python tools/bench_workloads.py models --steps 20 --warmup 3 > gpurun_out/r5_models_$mode.txt 2>&1 || exit $?
  echo "mode=$mode"; grep -o '"model": "[a-z0-9_]*", "ms_per_step": [0-9.]*' gpurun_out/r5_models_$mode.txt
done
for arch in campplus ecapa; do
  timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/r5_steps_${arch}_k.json > gpurun_out/r5_steps_${arch}_k.txt 2>&1 || exit $?
  echo "$arch $(grep -v amdgpu.ids gpurun_out/r5_steps_${arch}_k.txt | head -1)"
done
