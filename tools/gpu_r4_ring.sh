#!/bin/bash
# Round 4: golden tests of the LDS-DMA ring GEMM, then an A/B against the register-staged GEMM.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest $(date +%T)"
timeout -k 10 420 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_c2_full.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ring.log 2>&1
rc=$?; tail -5 gpurun_out/pt_ring.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
LIBS="3d-speaker_amd/lib/libspk_hip.so:SPK_RING=0 3d-speaker_amd/lib/libspk_hip.so" REPS=${REPS:-2} ARCHS=${ARCHS:-"eres2netv2 eres2net_large"} bash tools/gpu_ab.sh
