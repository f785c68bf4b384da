#!/bin/bash
# Quick GPU iteration: model parity tests + per-step profile of one arch (+ optional extra arch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
arch=${1:-eres2netv2}
echo "== pytest models $(date +%T)"
timeout -k 10 600 python -m pytest tests/test_gpu_models.py tests/test_gpu_fbank.py -q -x -rf > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_quick.log
if [ $rc -ne 0 ]; then exit $rc; fi
for a in $arch ${2:-}; do
  echo "== steps $a $(date +%T)"
  timeout -k 10 300 python tools/profile_steps.py --arch $a --json gpurun_out/steps_$a.json > gpurun_out/steps_$a.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/steps_$a.txt | head -3
  if [ $rc -ne 0 ]; then exit $rc; fi
  python tools/agg_steps.py gpurun_out/steps_$a.json | head -24
done
if [ -n "${CMP_F32:-}" ]; then
  echo "== steps $arch fp32-MFMA $(date +%T)"
  SPK_CONV_MFMA=f32 timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/steps_${arch}_f32.json > gpurun_out/steps_${arch}_f32.txt 2>&1
  grep -v amdgpu.ids gpurun_out/steps_${arch}_f32.txt | head -2
  python tools/agg_steps.py gpurun_out/steps_${arch}_f32.json | head -16
fi
