#!/bin/bash
# rocprofv3 --kernel-trace --stats of one per-step profile per model (tools/profile_steps.py),
# outputs gpurun_out/pm_<arch>/ (each step under its own time limit; stop at the first failure)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in ${ARCHS:-eres2net_large ecapa campplus}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pm_$a -o run --output-format csv -- \
      python tools/profile_steps.py --arch $a > gpurun_out/pm_$a.log 2>&1 || exit $?
  echo "$a: $(grep -v amdgpu.ids gpurun_out/pm_$a.log | grep ms/forward | head -1)"
done
