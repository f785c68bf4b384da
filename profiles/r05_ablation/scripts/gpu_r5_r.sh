#!/bin/bash
# round-5 GPU pass R: 64x32 tiles for the N <= 32 GEMMs (CAM++ CAM local convs) and the fused
# CAM segment-sum + gate kernel: tests, timings (SPK_CAM_GATE_PAIR=1: the two-launch pair)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_range_guard.py tests/test_gpu_c3_full.py tests/test_gpu_precision_fp16.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_n32_tests.log 2>&1 || { tail -30 gpurun_out/r5_n32_tests.log; exit 1; }
tail -1 gpurun_out/r5_n32_tests.log
timeout -k 10 300 python tools/profile_steps.py --arch campplus --json gpurun_out/r5_steps_campplus_r.json > gpurun_out/r5_steps_campplus_r.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5_steps_campplus_r.txt | head -1
python - <<PY
import json
from collections import defaultdict
d = defaultdict(lambda: [0, 0.0])
for x in json.load(open('gpurun_out/r5_steps_campplus_r.json')):
    d[x['kernel']][0] += 1; d[x['kernel']][1] += x['ms']
for k, v in sorted(d.items(), key=lambda t: -t[1][1])[:4]: print(f'{v[0]:4d} {v[1]:.3f} {k}')
PY
SPK_CAM_GATE_PAIR=1 timeout -k 10 300 python tools/profile_steps.py --arch campplus > gpurun_out/r5_steps_campplus_pair.txt 2>&1 || exit $?
echo "pair: $(grep -v amdgpu.ids gpurun_out/r5_steps_campplus_pair.txt | head -1)"
for w in c3 "c3 --precision fp16" models; do
  timeout -k 10 300 python tools/bench_workloads.py $w 2>/dev/null | grep -o '"model": "[a-z0-9_+()A-Z]*", [^}]*"ms_per_step": [0-9.]*' | head -4
done
