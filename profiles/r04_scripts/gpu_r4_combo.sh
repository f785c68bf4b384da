#!/bin/bash
# Round 4 combined call (the pool's slots are scarce): goldens + range guard of the in-tree
# library, per-step A/B against ab/libspk_head.so, then tools/gpu_r4_misc.sh (memset probe,
# AFF residency A/B, secondary workloads).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== goldens $(date +%T)"
timeout -k 10 420 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_c2_full.py tests/test_gpu_range_guard.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_models.log 2>&1
rc=$?; tail -3 gpurun_out/pt_models.log; echo "goldens rc=$rc"
[ $rc -ne 0 ] && exit $rc
LIBS="3d-speaker_amd/lib/libspk_hip.so ab/libspk_head.so" REPS=1 ARCHS="eres2netv2 eres2net_large campplus" bash tools/gpu_ab.sh || exit $?
bash tools/gpu_r4_misc.sh
