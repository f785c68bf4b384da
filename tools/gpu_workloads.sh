#!/bin/bash
# Secondary BASELINE.json workloads on one GPU: C1, C3, all models at B=256, C4 (N=1), C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
for w in c1 c3 models; do
  echo "== $w $(date +%T)"
  timeout -k 10 300 python tools/bench_workloads.py $w > gpurun_out/wl_$w.json 2> gpurun_out/wl_$w.err
  rc=$?; cat gpurun_out/wl_$w.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/wl_$w.err; fi
  if fatal $rc; then exit $rc; fi
done
echo "== c3 fp16 mode $(date +%T)"
timeout -k 10 300 python tools/bench_workloads.py c3 --precision fp16 > gpurun_out/wl_c3_fp16.json 2> gpurun_out/wl_c3_fp16.err
rc=$?; cat gpurun_out/wl_c3_fp16.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/wl_c3_fp16.err; fi
if fatal $rc; then exit $rc; fi
echo "== c4 $(date +%T)"
timeout -k 10 400 python tools/bench_c4.py ${C4_ARGS:-} > gpurun_out/wl_c4.json 2> gpurun_out/wl_c4.err
rc=$?; cat gpurun_out/wl_c4.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/wl_c4.err; fi
if fatal $rc; then exit $rc; fi
echo "== c5 $(date +%T)"
timeout -k 10 500 python tools/bench_diarization.py ${C5_ARGS:-} > gpurun_out/wl_c5.json 2> gpurun_out/wl_c5.err
rc=$?; cat gpurun_out/wl_c5.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/wl_c5.err; fi
echo "== done $(date +%T)"
exit $rc
