#!/bin/bash
# Round 4 combined call: persistent ring GEMM goldens, A/B vs the register-staged GEMM and the
# non-persistent ablation builds, then the range-word reset probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest $(date +%T)"
timeout -k 10 420 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_c2_full.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ring.log 2>&1
rc=$?; tail -3 gpurun_out/pt_ring.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
LIBS="3d-speaker_amd/lib/libspk_hip.so 3d-speaker_amd/lib/libspk_hip.so:SPK_RING_GRID=0 3d-speaker_amd/lib/libspk_hip.so:SPK_RING=0 ab/libspk_r5.so ab/libspk_r6.so" REPS=1 ARCHS=eres2netv2 bash tools/gpu_ab.sh || exit $?
bash tools/gpu_r4_memset.sh
