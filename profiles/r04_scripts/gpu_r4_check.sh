#!/bin/bash
# Round 4 check of the current tree: model goldens first (fast fail), per-step A/B of the ring
# GEMM against the register-staged one, then smoke, the whole GPU suite and the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
echo "== goldens $(date +%T)"
timeout -k 10 420 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_c2_full.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_models.log 2>&1
rc=$?; tail -3 gpurun_out/pt_models.log; echo "goldens rc=$rc"
[ $rc -ne 0 ] && exit $rc
LIBS=${LIBS:-"3d-speaker_amd/lib/libspk_hip.so"} REPS=${REPS:-1} ARCHS=${ARCHS:-"eres2netv2"} bash tools/gpu_ab.sh || exit $?
[ "${QUICK:-0}" = "1" ] && exit 0
echo "== smoke $(date +%T)"
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
echo "== pytest -m gpu $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if fatal $rc; then exit $rc; fi
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-1200
echo "== done $(date +%T)"
exit $rc
