#!/bin/bash
# Round 4: goldens + range-guard tests of the current tree, per-step A/B of the operand split
# (fma_mix vs the round-3 form, ab/libspk_nomix.so), bench with the segmented guard vs the
# whole-plan twin (SPK_GUARD_SEGMENTS=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== goldens $(date +%T)"
timeout -k 10 420 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_c2_full.py tests/test_gpu_range_guard.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_models.log 2>&1
rc=$?; tail -3 gpurun_out/pt_models.log; echo "goldens rc=$rc"
[ $rc -ne 0 ] && exit $rc
L=3d-speaker_amd/lib/libspk_hip.so
LIBS=${LIBS:-"$L ab/libspk_nomix.so"} REPS=${REPS:-2} ARCHS=${ARCHS:-"eres2netv2 eres2net_large campplus"} bash tools/gpu_ab.sh || exit $?
for seg in 1 0; do
  echo "== bench SPK_GUARD_SEGMENTS=$seg $(date +%T)"
  SPK_GUARD_SEGMENTS=$seg timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_seg$seg.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_seg$seg.log | cut -c1-420
  [ $rc -ne 0 ] && exit $rc
done
exit 0
