#!/bin/bash
# Full GPU check: smoke, GPU tests, concurrency probes, MFMA counter pass, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
echo "== smoke $(date +%T)"
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
if fatal $rc; then exit $rc; fi
echo "== pytest -m gpu $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
if fatal $rc; then exit $rc; fi
echo "== concurrency probes $(date +%T)"
timeout -k 10 200 python tools/race_probe.py eres2netv2 3 2>&1 | grep -v amdgpu.ids | tail -2
rc=$?; if fatal $rc; then exit $rc; fi
timeout -k 10 200 python tools/race_probe3.py eres2netv2 2>&1 | grep -v amdgpu.ids | head -8
rc=$?; if fatal $rc; then exit $rc; fi
if [ "${PMC:-1}" = "1" ]; then
  echo "== pmc mfma $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma -o run --output-format csv -- python tools/profile_steps.py --arch eres2netv2 > gpurun_out/pmc_mfma.log 2>&1
  rc=$?; echo "pmc rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_mfma.log; exit $rc; fi
  python tools/pmc_mfma.py gpurun_out/pmc_mfma -o gpurun_out/sq_counters.json | head -16
fi
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400
echo "== done $(date +%T)"
exit $rc
