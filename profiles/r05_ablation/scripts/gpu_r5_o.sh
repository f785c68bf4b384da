#!/bin/bash
# round-5 GPU pass O: register-resident AFF (aff_x3r_kernel) vs aff_x3_kernel: goldens, per-step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_c2_full.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_aff_tests.log 2>&1 || { tail -40 gpurun_out/r5_aff_tests.log; exit 1; }
tail -2 gpurun_out/r5_aff_tests.log
for reg in 1 0 1 0; do
  SPK_AFF_REG=$reg timeout -k 10 300 python tools/profile_steps.py --arch eres2netv2 --json gpurun_out/r5_steps_aff$reg.json > gpurun_out/r5_steps_aff$reg.txt 2>&1 || exit $?
  python - <<PY
import json
a = json.load(open('gpurun_out/r5_steps_aff$reg.json'))
aff = [x for x in a if 'aff' in x['kernel']]
print('SPK_AFF_REG=$reg total %.3f ms, AFF %d launches %.3f ms' % (sum(x['ms'] for x in a), len(aff), sum(x['ms'] for x in aff)))
PY
done
