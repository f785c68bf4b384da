#!/bin/bash
# round-5 GPU pass G: 256x256 loop schedule variants; gated exact-twin cost per model
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=3d-speaker_amd/lib/libspk_hip.so
timeout -k 10 400 ./tools/gemm_bench --reps 10 --shapes l3.conv1,l3.conv3,l4.conv1,l4.conv3,l4.convs0,l3_ds \
  $L ablibs/libspk_sch1.so ablibs/libspk_sch2.so ablibs/libspk_sch3.so > gpurun_out/r5_sched.txt 2>&1 || exit $?
cat gpurun_out/r5_sched.txt
for rr in 0 1; do
  if [ $rr = 1 ]; then export SPK_DIAG_NO_RERUN=1; fi
  timeout -k 10 400 python tools/bench_workloads.py models --steps 20 --warmup 3 > gpurun_out/r5_models_norerun$rr.txt 2>&1 || exit $?
  echo "no_rerun=$rr"; grep -o '"model": "[a-z0-9_]*", "ms_per_step": [0-9.]*' gpurun_out/r5_models_norerun$rr.txt
done
