#!/bin/bash
# Round 4 diagnostics: phase stamps of the stage-1 fused block (ab/libspk_r2prof.so, built by
# tools/build_r2prof.sh) and ablation builds of the halo 3x3 kernel (SPK_EXP=1 no halo
# prefetch, 2 no epilogue, 3 no taps; tools/variant_lib.sh haloexpN) against the in-tree one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== r2 phase profile $(date +%T)"
SPK_HIP_LIB=ab/libspk_r2prof.so timeout -k 10 300 python tools/r2_prof.py > gpurun_out/r2_prof.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r2_prof.txt | tail -12; echo "r2 rc=$rc"
[ $rc -ne 0 ] && exit $rc
L=3d-speaker_amd/lib/libspk_hip.so
LIBS="$L ab/libspk_haloexp1.so ab/libspk_haloexp2.so ab/libspk_haloexp3.so" REPS=${REPS:-1} ARCHS=eres2netv2 bash tools/gpu_ab.sh
