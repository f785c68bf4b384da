#!/bin/bash
# Round 4: the captured-memset word reset probe (tools/gpu_r4_memset.sh), an AFF residency A/B
# (SPK_AFF_LDS_KB), then the secondary BASELINE workloads (C1, C3 in both modes, all models,
# C4, C5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
bash tools/gpu_r4_memset.sh > gpurun_out/memset_probe.log 2>&1
rc=$?; cat gpurun_out/memset_probe.log | grep -v amdgpu.ids | tail -40; echo "memset probe rc=$rc"
if fatal $rc; then exit $rc; fi
L=3d-speaker_amd/lib/libspk_hip.so
LIBS="$L $L:SPK_AFF_LDS_KB=50 $L:SPK_AFF_LDS_KB=40" REPS=1 ARCHS=eres2netv2 bash tools/gpu_ab.sh || exit $?
for w in "c1" "c3" "c3 --precision fp16" "models"; do
  tag=$(echo $w | tr -c 'a-z0-9\n' '_')
  echo "== workload $w $(date +%T)"
  timeout -k 10 300 python tools/bench_workloads.py $w > gpurun_out/wl_$tag.json 2> gpurun_out/wl_$tag.err
  rc=$?; head -c 700 gpurun_out/wl_$tag.json; echo; if [ $rc -ne 0 ]; then tail -5 gpurun_out/wl_$tag.err; fi
  if fatal $rc; then exit $rc; fi
done
echo "== c4 $(date +%T)"
timeout -k 10 400 python tools/bench_c4.py > gpurun_out/wl_c4.json 2> gpurun_out/wl_c4.err
rc=$?; head -c 700 gpurun_out/wl_c4.json; echo; if fatal $rc; then exit $rc; fi
echo "== c5 $(date +%T)"
timeout -k 10 500 python tools/bench_diarization.py > gpurun_out/wl_c5.json 2> gpurun_out/wl_c5.err
rc=$?; head -c 700 gpurun_out/wl_c5.json; echo
echo "== done $(date +%T)"
exit $rc
