#!/bin/bash
# round-5 GPU pass I: C5 full-size test, then the whole GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_full.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/r5_c5_full.log 2>&1 || { tail -30 gpurun_out/r5_c5_full.log; exit 1; }
grep -E "chunks|DER|passed|failed" gpurun_out/r5_c5_full.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_gputest_i.log 2>&1; rc=$?; tail -3 gpurun_out/r5_gputest_i.log; exit $rc
