#!/bin/bash
# Round 4: the captured memset-node word reset (SPK_WORD_RESET=memset) vs the kernel node,
# two forwards of one handle on two streams at once (tools/race_probe.py) and step bisection.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mode in kernel memset; do
  echo "== word reset: $mode $(date +%T)"
  if [ $mode = memset ]; then export SPK_WORD_RESET=memset; else unset SPK_WORD_RESET; fi
  timeout -k 10 240 python tools/race_probe.py eres2netv2 4 > gpurun_out/race_$mode.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/race_$mode.log | tail -14
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 240 python tools/race_probe2.py eres2netv2 > gpurun_out/race2_$mode.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/race2_$mode.log | tail -12
  [ $rc -ne 0 ] && exit $rc
done
exit 0
