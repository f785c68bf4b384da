#!/bin/bash
# GPU session: tests, per-step profiles of all four models, PMC traffic passes,
# rocprofv3 kernel stats, bench.  `prof` as $1 enables the rocprofv3 steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
echo "== pytest -m gpu $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
if fatal $rc; then exit $rc; fi
for a in eres2netv2 eres2net_large ecapa campplus; do
  echo "== steps $a $(date +%T)"
  timeout -k 10 300 python tools/profile_steps.py --arch $a --json gpurun_out/steps_$a.json > gpurun_out/steps_$a.txt 2>&1
  rc=$?; head -6 gpurun_out/steps_$a.txt
  if fatal $rc; then exit $rc; fi
done
if [ "${1:-}" = "prof" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== rocprofv3 --pmc $c $(date +%T)"
    timeout -k 10 600 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- \
        python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$c.log 2>&1
    rc=$?; echo "pmc rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$c.log; exit $rc; fi
  done
  python tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE -o gpurun_out/pmc_traffic.json \
      && cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
  echo "== rocprofv3 stats $(date +%T)"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-900
echo "== done $(date +%T)"
exit $rc
