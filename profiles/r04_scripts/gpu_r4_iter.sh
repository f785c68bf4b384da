#!/bin/bash
# Round 4 iteration check: model goldens + range guard (fast fail), per-step timings of
# $ARCHS with the in-tree library, optional A/B libraries ($LIBS), bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== goldens $(date +%T)"
timeout -k 10 420 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_c2_full.py tests/test_gpu_range_guard.py ${EXTRA_TESTS:-} -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_models.log 2>&1
rc=$?; tail -3 gpurun_out/pt_models.log; echo "goldens rc=$rc"
[ $rc -ne 0 ] && exit $rc
LIBS=${LIBS:-"3d-speaker_amd/lib/libspk_hip.so"} REPS=${REPS:-1} ARCHS=${ARCHS:-"eres2netv2 campplus"} bash tools/gpu_ab.sh || exit $?
if [ "${BENCH:-1}" = "1" ]; then
  echo "== bench $(date +%T)"
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
fi
exit $rc
