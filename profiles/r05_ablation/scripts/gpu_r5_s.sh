#!/bin/bash
# round-5 GPU pass S: halo 3x3 kernel with the weights' hi plane in registers (default) vs LDS
# (ablibs/libspk_wreg0.so, SPK_HALO_WREG=0): goldens, then alternating per-step profiles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_wreg_tests.log 2>&1 || { tail -30 gpurun_out/r5_wreg_tests.log; exit 1; }
tail -1 gpurun_out/r5_wreg_tests.log
for rep in 1 2; do
  for arm in wreg1 wreg0; do
    lib=""; [ $arm = wreg0 ] && lib=ablibs/libspk_wreg0.so
    for arch in eres2netv2 campplus; do
      env ${lib:+SPK_HIP_LIB=$lib} timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/r5_steps_${arch}_${arm}_$rep.json > /dev/null 2>&1 || exit $?
      python - <<PY
import json
a = json.load(open('gpurun_out/r5_steps_${arch}_${arm}_$rep.json'))
h = [x for x in a if 'halo' in x['kernel']]
print('$arm rep $rep $arch: total %.3f ms, halo %d launches %.3f ms' % (sum(x['ms'] for x in a), len(h), sum(x['ms'] for x in h)))
PY
    done
  done
done
