#!/bin/bash
# A/B of builds of libspk_hip.so (SPK_HIP_LIB): per-forward time of each arch, alternating.
# LIBS="a.so b.so:VAR=val ..." (default: ab/libspk_head.so and the in-tree build), ARCHS, REPS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=${LIBS:-"ab/libspk_head.so 3d-speaker_amd/lib/libspk_hip.so"}
for arch in ${ARCHS:-eres2netv2 eres2net_large}; do
  for rep in $(seq 1 ${REPS:-2}); do
    for ent in $LIBS; do
      lib=${ent%%:*}; envs=""; [ "$ent" != "$lib" ] && envs=${ent#*:}; envs=${envs//,/ }
      tag=$(basename $lib .so)${envs:+_${envs//[^A-Za-z0-9]/}}
      env $envs SPK_HIP_LIB=$lib timeout -k 10 300 python tools/profile_steps.py --arch $arch --json gpurun_out/ab_${arch}_${tag}_${rep}.json > gpurun_out/ab_${arch}_${tag}_${rep}.txt 2>&1
      rc=$?; echo "$tag/$rep $(grep -v amdgpu.ids gpurun_out/ab_${arch}_${tag}_${rep}.txt | head -1)"
      if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_${arch}_${tag}_${rep}.txt; exit $rc; fi
    done
  done
done
