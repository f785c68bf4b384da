#!/bin/bash
# Round-3 GPU evidence pass: smoke, pytest -m gpu, per-step profiles of four models, PMC
# traffic (FETCH/WRITE, separate passes), MFMA/SQ counters, rocprofv3 kernel stats, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
echo "== smoke $(date +%T)"
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== pytest -m gpu $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if fatal $rc; then exit $rc; fi
for a in eres2netv2 eres2net_large ecapa campplus; do
  timeout -k 10 300 python tools/profile_steps.py --arch $a --json gpurun_out/steps_$a.json > gpurun_out/steps_$a.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/steps_$a.txt | head -1
  if fatal $rc; then exit $rc; fi
done
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== rocprofv3 --pmc $c $(date +%T)"
  timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$c.log 2>&1
  rc=$?; echo "pmc rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$c.log; exit $rc; fi
done
python tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE -o gpurun_out/pmc_traffic.json \
    && cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
echo "== pmc sq $(date +%T)"
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma -o run --output-format csv -- python tools/profile_steps.py --arch eres2netv2 > gpurun_out/pmc_mfma.log 2>&1
rc=$?; echo "pmc sq rc=$rc"
if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_mfma.log; exit $rc; fi
python tools/pmc_mfma.py gpurun_out/pmc_mfma -o gpurun_out/sq_counters.json | head -12
echo "== rocprofv3 stats $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-600
echo "== done $(date +%T)"
exit $rc
