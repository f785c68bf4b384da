#!/bin/bash
# One GPU-box session: smoke -> GPU tests -> bench (-> optional rocprofv3 profile).
# Every GPU step has its own time limit; a crash/abort/timeout (rc not 0/1) ends the run.
# usage: bash tools/gpu_check.sh [prof]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

echo "== smoke $(date +%T)"
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if fatal $rc; then exit $rc; fi

echo "== pytest -m gpu $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if fatal $rc; then exit $rc; fi

echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
if fatal $rc; then exit $rc; fi

if [ "${1:-}" = "prof" ]; then
  echo "== rocprofv3 $(date +%T)"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof.log
fi
echo "== done $(date +%T)"
