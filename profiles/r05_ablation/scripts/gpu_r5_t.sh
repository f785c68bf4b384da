#!/bin/bash
# round-5 GPU pass T: AFF kernel residency -- chunk-operand ring (default) vs one chunk at a time
# (ablibs/libspk_noring.so, 118 VGPRs), each with the 60 KB LDS residency cap and with 19 KB
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in ring:60 ring:19 noring:60 noring:19; do
    lib=""; [ ${arm%%:*} = noring ] && lib=ablibs/libspk_noring.so
    for arch in eres2netv2 eres2net_large; do
      env ${lib:+SPK_HIP_LIB=$lib} SPK_AFF_LDS_KB=${arm##*:} timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/r5_aff_${arch}_${arm/:/_}_$rep.json > /dev/null 2>&1 || exit $?
      python - <<PY
import json
a = json.load(open('gpurun_out/r5_aff_${arch}_${arm/:/_}_$rep.json'))
h = [x for x in a if 'aff' in x['kernel']]
print('$arm rep $rep $arch: total %.3f ms, AFF %d launches %.3f ms' % (sum(x['ms'] for x in a), len(h), sum(x['ms'] for x in h)))
PY
    done
  done
done
