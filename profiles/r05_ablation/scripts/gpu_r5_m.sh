#!/bin/bash
# round-5 GPU pass M: scaled split A/B (HEAD build vs two-instance kernels) on the ECAPA / CAM++
# and ERes2Net GEMM shapes, range-guard + model tests, model forwards scaled vs twin
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
timeout -k 10 400 ./tools/gemm_bench --reps 20 --shapes ec.b0,ec.r2n,ec.tdnn1,cam.transit,cam.linear1,l3.conv1,l4.convs0,l3_ds,l2.conv1 \
  ablibs/libspk_head.so $L > gpurun_out/r5_scaled_ab.txt 2>&1 || { cat gpurun_out/r5_scaled_ab.txt; exit 1; }
cat gpurun_out/r5_scaled_ab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_range_guard.py tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_scaled_tests.log 2>&1 || { tail -40 gpurun_out/r5_scaled_tests.log; exit 1; }
tail -2 gpurun_out/r5_scaled_tests.log
for mode in scaled twin; do
  SPK_RANGE_MODE=$mode timeout -k 10 400 python tools/bench_workloads.py models --steps 20 --warmup 3 > gpurun_out/r5_models_$mode.txt 2>&1 || exit $?
  echo "mode=$mode"; grep -o '"model": "[a-z0-9_]*", "ms_per_step": [0-9.]*' gpurun_out/r5_models_$mode.txt
done
