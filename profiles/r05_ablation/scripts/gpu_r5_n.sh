#!/bin/bash
# round-5 GPU pass N: the captured guarded forward's graph (hipGraphDebugDotPrint) for the
# memset-node and kernel-node word resets, then the two-stream race probe once per arm
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SPK_WORD_RESET=memset SPK_GRAPH_DOT=gpurun_out/g_memset.dot timeout -k 10 240 python tools/graph_dot_probe.py > gpurun_out/r5_dot.log 2>&1 || { cat gpurun_out/r5_dot.log; exit 1; }
SPK_GRAPH_DOT=gpurun_out/g_kernel.dot timeout -k 10 240 python tools/graph_dot_probe.py >> gpurun_out/r5_dot.log 2>&1 || { cat gpurun_out/r5_dot.log; exit 1; }
python tools/graph_dot_probe.py --parse gpurun_out/g_memset.dot gpurun_out/g_kernel.dot >> gpurun_out/r5_dot.log 2>&1
grep -v amdgpu.ids gpurun_out/r5_dot.log
for mode in kernel memset; do
  echo "== word reset: $mode"
  if [ $mode = memset ]; then export SPK_WORD_RESET=memset; else unset SPK_WORD_RESET; fi
  timeout -k 10 240 python tools/race_probe.py eres2netv2 4 > gpurun_out/r5_race_$mode.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r5_race_$mode.log | tail -10
done
